#!/bin/bash
# Round-6 GPU checks, stage by stage (STAGES="tests rehearse bench ..." selects).  Every GPU
# step has its own time limit; a fault, abort or timeout stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <limit_s> <cmd...>   (stdout/err -> gpurun_out/<name>.log)
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s): $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
for s in ${STAGES:-xtests bench}; do
  case $s in
    xtests)  # the exchange: in-process sharded ranks, bitwise cross-transport, self-test fallback
      step xtests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
        tests/test_sharded_inproc_gpu.py tests/test_peer_allreduce_gpu.py ;;
    bn)  # BatchNorm fixed-point statistics
      step bntests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
        tests/test_hip_ops_gpu.py tests/test_conv_gemm_gpu.py -k "bn or bnin" ;;
    tests)
      step gputests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    bench)
      step bench_n1 200 python bench.py --gpus 1 --steps 20 --warmup 5
      step bench_n1b 200 python bench.py --gpus 1 --steps 20 --warmup 5
      step bench_n1_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 ;;
    rehearse)  # the driver's multi-GPU launch, N ranks sharing cuda:0 (gloo control plane)
      for N in ${RANKS:-2}; do
        DAMD_COMM=gloo step share_n$N 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
          --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 200 --warmup 20
      done ;;
    fused)
      step fused 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_convnet_gpu.py ;;
    bextra)  # the bench's window repeated (stderr): first-window vs steady cost at K = 20
      DAMD_BENCH_EXTRA=3 step bench_extra 200 python bench.py --gpus 1 --steps 20 --warmup 5
      DAMD_GRAPH_STEPS=5 DAMD_BENCH_EXTRA=3 step bench_extra_g5 200 python bench.py --gpus 1 --steps 20 --warmup 5
      DAMD_BENCH_EXTRA=3 step bench_extra_b 200 python bench.py --gpus 1 --steps 20 --warmup 5
      DAMD_GRAPH_STEPS=5 DAMD_BENCH_EXTRA=3 step bench_extra_g5b 200 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    ab)  # same-box A/B: build/ab/A (scripts/ab_build.sh) against the working tree, alternating
      for i in 1 2 3; do
        step ab_A_long$i 200 bash -c "cd build/ab/A && python bench.py --gpus 1 --steps 2000 --warmup 200"
        step ab_B_long$i 200 python bench.py --gpus 1 --steps 2000 --warmup 200
        step ab_A_short$i 200 bash -c "cd build/ab/A && python bench.py --gpus 1 --steps 20 --warmup 5"
        step ab_B_short$i 200 python bench.py --gpus 1 --steps 20 --warmup 5
      done ;;
    ppsweep)  # slice sizes: fwd positions per block (DAMD_PP) x bwd (DAMD_PP_BWD), long runs
      for pp in 2 3 4; do for pb in 1 2 3; do
        DAMD_PP=$pp DAMD_PP_BWD=$pb step pp_${pp}_${pb} 200 python bench.py --gpus 1 --steps 2000 --warmup 200
      done; done ;;
    ovh)  # fixed cost of a timed window (launch, flush, sync): fit over K
      step overhead 300 python scripts/overhead_probe.py ;;
    stamps)
      step stamps 200 python scripts/stamps.py 64 ;;
    gprobe)
      step gprobe 300 python scripts/probe_graph_branches.py 4 8 ;;
    dpprof)  # ResNet-18 N = 2 sharing the GPU: bucket all-reduce overlap (peer transport)
      step dpprof 500 bash scripts/prof_resnet_dp.sh
      python scripts/dp_overlap.py gpurun_out/prof_rn_dp/rn_kernel_trace.csv gpurun_out/dp_overlap.txt || true ;;
    ngpeer)
      step ngpeer 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_peer_allreduce_gpu.py -k native_graph ;;
    c3)  # direct conv kernels on the ResNet-18 shapes
      step c3base 300 python scripts/conv3_probe.py 64 ;;
    mab)  # MNIST step A/B on one box: prefetch + parity hints on / off, alternating
      for i in 1 2; do
        step mab_on$i 200 python bench.py --gpus 1 --steps 20 --warmup 5
        DAMD_XPREFETCH=0 DAMD_PAR_HINT=0 step mab_off$i 200 python bench.py --gpus 1 --steps 20 --warmup 5
      done
      step mab_on_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200
      DAMD_XPREFETCH=0 DAMD_PAR_HINT=0 step mab_off_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200
      DAMD_XPREFETCH=0 DAMD_PAR_HINT=0 step stamps_off 200 python scripts/stamps.py 64
      step stamps_on 200 python scripts/stamps.py 64 ;;
    shdiag)  # the sharded exchange at N = 2 sharing the GPU: pinned, with / without the self-test
      DAMD_COMM=gloo DAMD_ALLREDUCE=sharded step sh_pinned 300 python bench.py --gpus 2 --steps 200 --warmup 20
      DAMD_COMM=gloo DAMD_ALLREDUCE=sharded DAMD_XCHG_SELFTEST=0 step sh_noself 300 python bench.py --gpus 2 --steps 200 --warmup 20
      DAMD_COMM=gloo DAMD_ALLREDUCE=xgmi step xg_pinned 300 python bench.py --gpus 2 --steps 200 --warmup 20 ;;
    c3r)  # the persistent 64 -> 64 direct conv (conv3r.hip) and every direct-conv test
      step c3r 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py -k "conv3" ;;
    c3ab)  # direct conv kernels on the ResNet-18 shapes, conv3r on / off
      DAMD_CONV3R=1 step c3ab_on 300 python scripts/conv3_probe.py 64
      DAMD_CONV3R=0 step c3ab_off 300 python scripts/conv3_probe.py 64 ;;
    abt)  # one GPU test in the round-5 tree (build/ab/A) and in the working tree
      K=${ABT_K:-short_final_batch}
      (cd build/ab/A && timeout -k 10 200 python -u -m pytest -q -p no:cacheprovider tests/test_native_graph_gpu.py -k "$K" -s) > gpurun_out/abt_A.log 2>&1; echo "abt_A rc=$?"; tail -5 gpurun_out/abt_A.log
      timeout -k 10 200 python -u -m pytest -q -p no:cacheprovider tests/test_native_graph_gpu.py -k "$K" -s > gpurun_out/abt_B.log 2>&1; echo "abt_B rc=$?"; tail -5 gpurun_out/abt_B.log ;;
    peer)  # the multi-rank exchange tests (ranks sharing the GPU)
      step peer 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_peer_allreduce_gpu.py ;;
    testsall)  # every GPU test, no -x: all failures at once
      timeout -k 10 1300 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/testsall.log 2>&1
      rc=$?; echo "testsall rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/testsall.log | tail -20
      if [ $rc -gt 1 ]; then exit $rc; fi ;;
    c3s)  # the strip kernel's correctness first (its own limit), then timings
      step c3s 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gemm_gpu.py -k "conv3r" ;;
    pmc)  # PMC passes per direct-conv mode (one shape each)
      for cfg in "l1f:56 64 64 fwd" "l1d:56 64 64 dgrad" "l2f:28 128 128 fwd" "l3f:14 256 256 fwd" "l3d:14 256 256 dgrad" "l1w:56 64 64 wgrad"; do
        TAG=${cfg%%:*} CONV="${cfg#*:}" step pmc_${cfg%%:*} 200 bash scripts/pmc_conv.sh
      done ;;
    ngraph)  # bucket graph structure + native-graph tests
      step ngraph 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_native_graph_gpu.py ;;
    resnet)
      step resnet 300 python bench.py --model resnet18 --steps 20 --warmup 5
      step resnet_long 300 python bench.py --model resnet18 --steps 100 --warmup 10 ;;
    bnab)  # bn_bwd_reduce grid size A/B (fixed-point accumulator atomics vs memory parallelism)
      for t in 1024 512 256; do
        DAMD_BN_BWD_BLOCKS=$t step rn_bnt$t 300 python bench.py --model resnet18 --steps 50 --warmup 10
      done ;;
    rnprof)
      step rnprof 400 bash scripts/prof_resnet.sh ;;
    wsprof)  # kernel trace of the step with the weight-gradient side stream on
      DAMD_WGRAD_STREAM=1 PROF_OUT=gpurun_out/prof_rn_ws step wsprof 400 bash scripts/prof_resnet.sh
      PROF_OUT=gpurun_out/prof_rn_base step rnprof_base 400 bash scripts/prof_resnet.sh ;;
    rnab)  # ResNet-18 step, build/ab/A (scripts/ab_build.sh) against the working tree, alternating
      for i in 1 2 3; do
        step rnab_A$i 300 bash -c "cd build/ab/A && python bench.py --model resnet18 --steps 50 --warmup 10"
        step rnab_B$i 300 python bench.py --model resnet18 --steps 50 --warmup 10
      done
      grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/rnab_A*.log gpurun_out/rnab_B*.log ;;
    bngrid)  # BN kernel grids: minimum KiB per block (apply with finalize / backward reduce)
      for cfg in "0 0" "32 0" "64 0" "0 32" "0 64" "32 32" "0 0"; do
        set -- $cfg
        DAMD_BN_FIN_MINKB=$1 DAMD_BN_BWD_MINKB=$2 step bng_$1_$2 300 python bench.py --model resnet18 --steps 50 --warmup 10
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/bng_*.log ;;
    dual)  # dual-BN backward + the apply reading the masked gradient: bitwise tests
      step dual 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_native_graph_gpu.py \
        -k "dual or bitwise or short_final or one_step or emulated" ;;
    stem)  # stem BN/ReLU/MaxPool kernels: numerics, then the step with the stem reduce grid swept
      step stemt 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_ops_gpu.py \
        tests/test_native_graph_gpu.py tests/test_conv_gemm_gpu.py -k "pool or stem or maxpool" ;;
    stemab)
      for i in 1 2; do
        step stab_A$i 300 bash -c "cd build/ab/A && python bench.py --model resnet18 --steps 50 --warmup 10"
        step stab_B$i 300 python bench.py --model resnet18 --steps 50 --warmup 10
        DAMD_POOL_BN_BLOCKS=1024 step stab_B1024_$i 300 python bench.py --model resnet18 --steps 50 --warmup 10
        DAMD_POOL_BN_BLOCKS=2048 step stab_B2048_$i 300 python bench.py --model resnet18 --steps 50 --warmup 10
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/stab_*.log ;;
    profab)  # kernel traces of build/ab/A and the working tree
      step profA 400 bash -c "cd build/ab/A && PROF_OUT=\$GRAFT_REPO_ROOT/gpurun_out/prof_A bash scripts/prof_resnet.sh"
      PROF_OUT=gpurun_out/prof_B step profB 400 bash scripts/prof_resnet.sh ;;
    splitsw)  # split-K planner thresholds (minimum tiles to skip split-K / target workgroups)
      for cfg in "320 384" "100 384" "200 384" "320 256" "320 512" "320 768" "320 384"; do
        set -- $cfg
        DAMD_SPLIT_MIN_TILES=$1 DAMD_SPLIT_TARGET_WG=$2 step spl_$1_$2 300 python bench.py --model resnet18 --steps 50 --warmup 10
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/spl_*.log ;;
    epi)  # epilogue operand prefetch: every conv / GEMM numerics test, then the A/B
      step epit 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gemm_gpu.py \
        tests/test_hip_ops_gpu.py tests/test_native_graph_gpu.py -k "not full_size and not side_stream" ;;
    stemd)  # the direct stem forward: bitwise against the implicit GEMM, the stem tests
      step stemd 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py \
        -k "stem" ;;
    stemp)
      step stemp 200 python scripts/stem_probe.py 64 ;;
    bnsw)  # BN knobs after the finalize rework: replicas, backward-reduce grid, apply grid cap
      for cfg in "8 512 768" "4 512 768" "16 512 768" "8 1024 768" "8 256 768" "8 512 1536" "8 512 384" "8 512 768"; do
        set -- $cfg
        DAMD_BN_REPS=$1 DAMD_BN_BWD_BLOCKS=$2 DAMD_BN_FIN_GRID=$3 step bnsw_$1_$2_$3 300 python bench.py --model resnet18 --steps 50 --warmup 10
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/bnsw_*.log ;;
    mnistprof)  # MNIST: bench at the driver's flags + long, phase stamps, PMC issue mix
      step mb_n1 200 python bench.py --gpus 1 --steps 20 --warmup 5
      step mb_n1b 200 python bench.py --gpus 1 --steps 20 --warmup 5
      step mb_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200
      step mstamps 200 python scripts/stamps.py 64
      step mpmc 400 bash scripts/pmc_mnist.sh ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    fixup)  # in-launch split-K finish: equivalence tests, then every conv / graph test
      step fixt 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gemm_gpu.py -k "splitk" &&
      step fixall 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gemm_gpu.py \
        tests/test_native_graph_gpu.py tests/test_native_layers_gpu.py -k "not full_size and not side_stream" ;;
    fixp)
      step fixp 200 python scripts/fixup_probe.py ;;
    rehx)  # N = 2 sharing the GPU: auto twice, peer pinned, sharded pinned
      for v in auto1 xgmi auto2 sharded; do
        DAMD_ALLREDUCE=${v%[12]} DAMD_COMM=gloo step rehx_$v 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 200 --warmup 20
      done ;;
    rehab)  # N = 2 sharing the GPU, peer pinned: build/ab/A against the working tree, alternating
      for i in 1 2; do
        DAMD_ALLREDUCE=xgmi DAMD_COMM=gloo step rehab_A$i 400 bash -c "cd build/ab/A && python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 200 --warmup 20"
        DAMD_ALLREDUCE=xgmi DAMD_COMM=gloo step rehab_B$i 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 2 --steps 200 --warmup 20
      done ;;
    bnall)  # every BN kernel test + the native-graph BN / dual / bitwise tests
      step bnall 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hip_ops_gpu.py \
        tests/test_native_graph_gpu.py tests/test_conv_gemm_gpu.py -k "bn or dual or bitwise or stem or emulated or one_step" ;;
    wstest)  # weight gradients on a side stream: bitwise against the single-stream step
      step wstest 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_native_graph_gpu.py -k side_stream ;;
    wsab)  # ResNet-18 step, weight-gradient side stream off / on / on for >= 128 outputs, alternating
      for i in 1 2; do
        DAMD_WGRAD_STREAM=0 step ws_off$i 300 python bench.py --model resnet18 --steps 50 --warmup 10
        DAMD_WGRAD_STREAM=1 step ws_on$i 300 python bench.py --model resnet18 --steps 50 --warmup 10
        DAMD_WGRAD_STREAM=1 DAMD_WGRAD_STREAM_MINC=128 step ws_on128_$i 300 python bench.py --model resnet18 --steps 50 --warmup 10
      done ;;
  esac
done
echo stages-done
