# LDS-DMA tile configs on the Xception-41 b128 pointwise shapes (forward and input gradient)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
S="128,19,728,728,1,1,0;128,38,728,728,1,1,0;128,10,1536,1536,1,1,0;128,19,728,1024,1,1,0;128,38,256,728,1,1,0"
timeout -k 10 400 python dev/tools/cfg_ab.py --op fwd --shapes "$S" --cfgs 0,1,2,3,4,6,reg --rounds 2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06_xcfg.log || exit 1
timeout -k 10 400 python dev/tools/cfg_ab.py --op dgrad --shapes "$S" --cfgs 0,1,2,3,4,6,reg --rounds 2 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_xcfg.log
