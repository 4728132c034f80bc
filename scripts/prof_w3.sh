export TMPDIR=/tmp; mkdir -p gpurun_out
BENCH_W3_ONLY=v9s2w256 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w3 -o w3 -- python scripts/bench_wgrad3.py > gpurun_out/prof_w3.log 2>&1
