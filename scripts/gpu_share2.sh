export TMPDIR=/tmp; mkdir -p gpurun_out
for split in 0 1; do
DAMD_SHARED_CU_SPLIT=$split DAMD_COMM=gloo timeout -k 10 150 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951$split bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/share2_split$split.log 2>&1
rc=$?; echo "split=$split rc=$rc"; tail -1 gpurun_out/share2_split$split.log | cut -c1-260; [ $rc -ne 0 ] && exit $rc
done
DAMD_COMM=gloo DAMD_ALLREDUCE=xgmi DAMD_SHARED_CU_SPLIT=1 timeout -k 10 150 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/share2x.log 2>&1
echo "xgmi rc=$?"; tail -1 gpurun_out/share2x.log | cut -c1-260
