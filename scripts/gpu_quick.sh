#!/bin/bash
# Quick GPU iteration: GPU tests (no -x), phase stamps, short bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/stamps.py 64 > gpurun_out/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 3000 --warmup 300 > gpurun_out/bench_n1.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
