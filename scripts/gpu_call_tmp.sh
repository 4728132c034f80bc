set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fused_convnet_gpu.py tests/test_sharded_inproc_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t_sel.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t_sel.log | head -20; tail -2 gpurun_out/t_sel.log
[ $rc -le 1 ] || exit $rc
for p in 1 0 1 0; do
  DAMD_CONV_SLAB=$p timeout -k 10 120 python -u bench.py > gpurun_out/slab_$p.log 2>&1 || exit 1
  echo "slab $p long: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/slab_$p.log)"
  DAMD_CONV_SLAB=$p timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/slabd_$p.log 2>&1 || exit 1
  echo "slab $p driver: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/slabd_$p.log)"
done
