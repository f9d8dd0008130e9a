# Stem pool kernels at the bench batch (1024): window loads up front vs the per-tap loop
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for v in 1 0 1 0; do
echo "TDL_POOL_PRELOAD=$v"
TDL_POOL_PRELOAD=$v timeout -k 10 120 python dev/tools/pool_bench.py --n 1024 --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
done
