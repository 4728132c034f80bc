set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gemm_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_conv.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t_conv.log)"; [ $rc -le 1 ] || exit $rc
DAMD_CONV3_HB2=0 timeout -k 10 300 python -u -m pytest tests/test_conv_gemm_gpu.py -q -x --timeout 200 --timeout-method thread -k conv3 > gpurun_out/t_conv0.log 2>&1
rc=$?; echo "tests hb2=0 rc=$rc: $(tail -1 gpurun_out/t_conv0.log)"; [ $rc -le 1 ] || exit $rc
for hb in 1 0; do for a in "28 128 128" "14 256 256" "14 256 256 dgrad" "28 128 128 dgrad"; do
  echo "hb2=$hb $a"; DAMD_CONV3_HB2=$hb timeout -k 10 120 python -u scripts/stamps_conv3.py $a 2>&1 | grep -E "blocks|taps|block total" || exit 1
done; done
for hb in 1 0 1; do
  DAMD_CONV3_HB2=$hb timeout -k 10 200 python -u bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/rn_hb$hb.log 2>&1 || exit $?
  echo "resnet hb2=$hb: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn_hb$hb.log)"
done
