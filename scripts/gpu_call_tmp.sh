set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 360 python -u scripts/diag_fold.py > gpurun_out/diag_fold.log 2>&1; echo "diag rc=$?"; grep -v INFO gpurun_out/diag_fold.log | tail -20
timeout -k 10 400 python -u -m pytest tests/test_peer_allreduce_gpu.py tests/test_sharded_inproc_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t_peer.log 2>&1; rc=$?; echo "peer tests rc=$rc"; tail -3 gpurun_out/t_peer.log
[ $rc -le 1 ] || exit $rc
bash scripts/prof_resnet.sh || exit 1
bash scripts/prof_resnet_dp.sh || exit 1
bash scripts/gpu_envprobe.sh || exit 1
