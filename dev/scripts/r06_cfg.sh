# LDS-DMA tile configs on the ResNet-50 b1024 1x1 shapes (forward and input gradient)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
S="1024,14,256,1024,1,1,0;1024,28,128,512,1,1,0;1024,7,512,2048,1,1,0;1024,7,2048,512,1,1,0;1024,14,1024,256,1,1,0;1024,56,64,256,1,1,0;1024,28,512,128,1,1,0;1024,56,256,64,1,1,0"
timeout -k 10 400 python dev/tools/cfg_ab.py --op fwd --shapes "$S" --cfgs 0,2,3,4,6 --rounds 2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06_cfg.log || exit 1
timeout -k 10 400 python dev/tools/cfg_ab.py --op dgrad --shapes "$S" --cfgs 0,2,3,4,6 --rounds 2 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_cfg.log
