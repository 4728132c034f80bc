set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_driver.log
done
timeout -k 10 200 python -u bench.py > gpurun_out/bench_long.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_long.log
