set -u
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 env DAMD_CONV_STAGES=3 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py > gpurun_out/t_st3.log 2>&1 || { tail -20 gpurun_out/t_st3.log; exit 1; }
tail -2 gpurun_out/t_st3.log
timeout -k 10 400 env BENCH_CFG=0:2,0:3,32:2,32:3,64:3 python -u scripts/bench_gemm.py > gpurun_out/bench_st.log 2>&1
