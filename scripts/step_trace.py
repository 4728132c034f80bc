import csv, sys
path, anchor, out = sys.argv[1], sys.argv[2], sys.argv[3]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if anchor in r['Kernel_Name']]
i, j = idx[-3], idx[-2]
t0 = int(rows[i]['Start_Timestamp']); busy = 0
with open(out, 'w') as f:
    f.write("start_us  dur_us  workgroups  kernel\n")
    for r in rows[i:j]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp']); busy += e - s
        # rocprofv3 reports the grid in work-items per dimension: workgroups = product over
        # X, Y AND Z (split-K launches put their slabs in Z)
        gx, gy, gz = (int(r.get(f'Grid_Size_{d}') or 1) for d in 'XYZ')
        bx, by, bz = (int(r.get(f'Workgroup_Size_{d}') or 1) for d in 'XYZ')
        wg = (gx // max(1, bx)) * (gy // max(1, by)) * (gz // max(1, bz))
        f.write(f"{(s-t0)/1000:8.1f} {(e-s)/1000:7.1f} {wg:10d}  {r['Kernel_Name'][:90]}\n")
    f.write(f"busy {busy/1000:.1f} us, span {(int(rows[j]['Start_Timestamp'])-t0)/1000:.1f} us\n")
