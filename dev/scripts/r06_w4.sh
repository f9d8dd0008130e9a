# 256x128 tiles on 4 waves of 128x64 (cfg 8) vs the 8-wave default (cfg 0): 1x1 forward and wgrad
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
S="1024,14,256,1024,1,1,0;1024,28,128,512,1,1,0;1024,7,512,2048,1,1,0;1024,7,2048,512,1,1,0;1024,14,1024,256,1,1,0;1024,56,64,256,1,1,0;1024,28,512,128,1,1,0;1024,56,256,64,1,1,0"
timeout -k 10 300 python dev/tools/cfg_ab.py --op fwd --shapes "$S" --cfgs 0,8 --rounds 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06_w4.log || exit 1
W="14,256,1024,1,1,0;28,128,512,1,1,0;7,512,2048,1,1,0;7,2048,512,1,1,0;14,1024,256,1,1,0;56,64,256,1,1,0;28,512,128,1,1,0;14,256,256,3,1,1"
timeout -k 10 400 python dev/tools/wgrad_ab.py --batch 1024 --rounds 3 --shapes "$W" --variants default,glds0,glds8 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_w4.log
