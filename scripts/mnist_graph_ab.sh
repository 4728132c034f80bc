# MNIST at the driver's flags: hipGraph (default) vs eager launches, alternating arms
set -o pipefail
for rep in 1 2 3; do
  for g in 1 0; do
    echo -n "DAMD_GRAPH=$g: " >> gpurun_out/mnist_graph_ab.log
    DAMD_GRAPH=$g timeout -k 10 120 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step']*1000)" >> gpurun_out/mnist_graph_ab.log || exit 1
  done
done
