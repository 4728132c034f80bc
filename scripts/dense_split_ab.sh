# ResNet-18 step with the classifier GEMMs split-K to 128 / 64 / 256 workgroups vs unsplit (1),
# alternating arms on one box
set -o pipefail
for rep in 1 2; do
  for wg in 128 1 64 256; do
    echo -n "DENSE_SPLIT_WG=$wg: " >> gpurun_out/dense_split_ab.log
    DAMD_DENSE_SPLIT_WG=$wg timeout -k 10 200 python bench.py --model resnet18 --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])" >> gpurun_out/dense_split_ab.log || exit 1
  done
done
