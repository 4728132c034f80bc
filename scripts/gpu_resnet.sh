#!/bin/bash
# ResNet-18 path on one GPU: kernel + engine tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own limit; any failure stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <limit_s> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -n 6
  [ $rc -eq 0 ] || exit $rc
}
run t_resnet 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_graph_gpu.py tests/test_conv_gemm_gpu.py tests/test_hip_ops_gpu.py
run bench_resnet 300 python -u bench.py --model resnet18 --steps 20 --warmup 5
run prof_resnet 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet4 -o resnet -- python bench.py --model resnet18 --steps 10 --warmup 3
echo resnet-done
