set -o pipefail
for wg in 256 512 384; do
  echo "== WG $wg" >> gpurun_out/wgsweep_probe.log
  DAMD_WGRAD3_WG=$wg timeout -k 10 120 python -u scripts/wgrad3_probe.py 3 >> gpurun_out/wgsweep_probe.log 2>&1 || exit 1
done
for rep in 1 2; do
  for wg in 256 512 384; do
    echo -n "WG $wg: " >> gpurun_out/wgsweep_bench.log
    DAMD_WGRAD3_WG=$wg timeout -k 10 200 python bench.py --model resnet18 --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])" >> gpurun_out/wgsweep_bench.log || exit 1
  done
done
