#!/bin/bash
# Full GPU check of the tree as the driver runs it: GPU tests, smoke(), the headline
# bench with the driver's flags and with defaults, the ResNet-18 bench, phase splits of
# both steps, and a rocprofv3 kernel-stats pass over the headline bench.  Every GPU step
# has its own time limit; test failures are reported and the benches still run, anything
# else (crash, abort, time limit) stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/pytest_gpu.log; exit $rc; fi  # a hang / crash stops here
tail -3 gpurun_out/pytest_gpu.log
step smoke 300 python -u __graft_entry__.py smoke
step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
tail -1 gpurun_out/bench_driver.log
step bench_default 300 python -u bench.py --phases 50
tail -1 gpurun_out/bench_default.log
step bench_resnet 300 python -u bench.py --model resnet18 --steps 20 --warmup 5 --phases 5
tail -1 gpurun_out/bench_resnet.log
step prof_mnist 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mnist -o bench -- python3 bench.py --gpus 1 --steps 500 --warmup 50
