set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_hip_ops_gpu.py > gpurun_out/t_conv.log 2>&1
rc=$?; tail -5 gpurun_out/t_conv.log; [ $rc -ne 0 ] && exit $rc
BENCH_CFG=0:2 timeout -k 10 240 python -u scripts/bench_gemm.py 64 > gpurun_out/bench_gemm2.log 2>&1; rc=$?; cat gpurun_out/bench_gemm2.log | grep -v amdgpu.ids; exit $rc
