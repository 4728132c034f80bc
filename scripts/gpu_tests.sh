#!/bin/bash
# Selected GPU test files (TESTS="tests/a.py tests/b.py"), then the driver's 1-GPU bench.
# Every GPU step has its own limit; a crash / abort / timeout stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${LIMIT:-600} python -u -m pytest ${TESTS:-tests} -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_sel.log | tail -8
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_sel.log; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_sel.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_sel.log; exit $rc
fi
