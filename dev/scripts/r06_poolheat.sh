# Stem pool kernels: isolated vs after a GEMM burst (power state), and the bench's own stem tensors
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python dev/tools/pool_bench.py > gpurun_out/poolh.log 2>&1 || exit $?
timeout -k 10 180 python dev/tools/pool_bench.py --heat --iters 10 >> gpurun_out/poolh.log 2>&1 || exit $?
cat gpurun_out/poolh.log
