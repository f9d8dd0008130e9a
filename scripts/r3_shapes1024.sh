# round 3: per-shape kernel A/B at the bench batch (1024): 3x3 weight gradients and 64-channel 3x3 forward
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python tools/wgrad_ab.py --batch 1024 --rounds 3 \
  --shapes "56,64,64,3,1,1;28,128,128,3,1,1;56,128,128,3,2,1;14,256,256,3,1,1;7,512,512,3,1,1;56,256,64,1,1,0;28,512,128,1,1,0" \
  > gpurun_out/wgrad1024.log 2>&1 || exit $?
cat gpurun_out/wgrad1024.log
timeout -k 10 300 python tools/cfg_ab.py --op fwd --cfgs 0,1,2,4,5,reg --rounds 3 \
  --shapes "1024,56,64,64,3,1,1;1024,56,64,64,1,1,0;1024,56,256,64,1,1,0" > gpurun_out/fwd64_1024.log 2>&1 || exit $?
cat gpurun_out/fwd64_1024.log
echo done
