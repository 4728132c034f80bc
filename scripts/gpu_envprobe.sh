#!/bin/bash
# Driver-flag MNIST bench under HIP runtime wait / graph settings, A/B on one box.
export TMPDIR=/tmp; mkdir -p gpurun_out
one() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 100 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/envp_run.log 2>&1 || { tail -5 gpurun_out/envp_run.log; exit 1; }
  echo "$lab $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/envp_run.log)"
}
for r in $(seq ${REPS:-2}); do
  one base X=1
  one awt1000 ROC_ACTIVE_WAIT_TIMEOUT=1000
  one awt0 ROC_ACTIVE_WAIT_TIMEOUT=0
  one pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
  one pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
done
for r in $(seq ${REPS:-2}); do
  timeout -k 10 100 python -u scripts/bench_spin.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/envp_run.log 2>&1 || { tail -5 gpurun_out/envp_run.log; exit 1; }
  echo "spin $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/envp_run.log) $(grep -o 'hipSetDeviceFlags.*' gpurun_out/envp_run.log)"
done
