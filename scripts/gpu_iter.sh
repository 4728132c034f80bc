#!/bin/bash
# one GPU iteration: the GPU test suite (failures reported, the benches still run), the
# ResNet-18 and MNIST benches, a rocprofv3 kernel trace of the ResNet-18 step
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log || true; tail -1 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then tail -40 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/bench_resnet.log 2>&1 || { tail -20 gpurun_out/bench_resnet.log; exit 1; }
tail -1 gpurun_out/bench_resnet.log | cut -c1-400
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { tail -20 gpurun_out/bench_driver.log; exit 1; }
tail -1 gpurun_out/bench_driver.log | cut -c1-200
PROF_OUT=gpurun_out/prof_resnet timeout -k 10 300 bash scripts/prof_resnet.sh || exit 1
