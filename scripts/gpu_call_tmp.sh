set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_sharded_inproc_gpu.py tests/test_fused_convnet_gpu.py tests/test_peer_allreduce_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t_sel.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/t_sel.log; tail -2 gpurun_out/t_sel.log
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_driver.log
done
timeout -k 10 200 python -u bench.py > gpurun_out/bench_long.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_long.log
timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/bench_rn.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_rn.log
for p in 0 1 0 1; do
  DAMD_PROBE_HCONV=$p timeout -k 10 120 python -u bench.py > gpurun_out/probec_$p.log 2>&1 || exit 1
  echo "probe hconv $p: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/probec_$p.log)"
done
