# ResNet-18 step with the direct 3x3 weight gradient at pipeline depth 3 (default) vs 4,
# alternating arms on one box
set -o pipefail
for rep in 1 2 3; do
  for st in 3 4; do
    echo -n "STAGES=$st: " >> gpurun_out/w3stages_ab.log
    DAMD_WGRAD3_STAGES=$st timeout -k 10 200 python bench.py --model resnet18 --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])" >> gpurun_out/w3stages_ab.log || exit 1
  done
done
