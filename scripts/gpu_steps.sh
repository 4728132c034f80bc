#!/bin/bash
# Run named GPU steps with their own limits: `bash scripts/gpu_steps.sh name:limit:cmd ...`.
# rc 0 / 1 (test failures) go on; anything else (fault, abort, timeout) ends the script.
export TMPDIR=/tmp; mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; lim=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; grep -v -E "amdgpu.ids|^(RCCL|HIP|ROCm) version|^Hostname|^Librccl" "gpurun_out/$name.log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
