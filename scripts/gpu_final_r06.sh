#!/bin/bash
# End-of-round check on one MI355X: every GPU test, smoke(), the driver's bench commands.
# Every GPU step under its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $O/bench_mnist.jsonl || exit 1
done
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 2>/dev/null | tail -1 >> $O/bench_resnet.jsonl || exit 1
cut -c1-200 $O/bench_mnist.jsonl $O/bench_resnet.jsonl
exit $rc
