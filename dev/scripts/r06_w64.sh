# 56x56x64 3x3 weight gradient: register GEMM (default) vs the halo kernel after the swizzle change
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 200 python dev/tools/dgrad_rows.py --op wgrad --shape 1024,56,64,64,3,1,1 --rows wgrad.gemm,wgrad.halo.aligned,wgrad.halo.wide3x3 --rounds 4 --iters 5 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python dev/tools/dgrad_rows.py --op wgrad --shape 1024,28,128,128,3,1,1 --rows wgrad.gemm,wgrad.halo.aligned,wgrad.halo.wide3x3 --rounds 4 --iters 5 2>&1 | grep -v amdgpu.ids
