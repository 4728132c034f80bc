set -u
export TMPDIR=/tmp
for pp in 2 3 4; do
  DAMD_PP=$pp timeout -k 10 120 python -u bench.py > gpurun_out/ab_pp$pp.log 2>&1 || exit 1
  echo "PP=$pp $(tail -1 gpurun_out/ab_pp$pp.log | cut -c1-160)"
done
