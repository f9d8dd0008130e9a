# round-5 final validation: the driver's tiers (GPU suite, smoke, dp2 rehearsal, bench) and the
# ResNet-152 fp8 vs bf16 pair on the same box
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash dev/scripts/gpu_r05final.sh
: > gpurun_out/final_r152.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/fp8  /' >> gpurun_out/final_r152.log
  timeout -k 10 300 python bench.py --model resnet152 --batch 256 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/bf16 /' >> gpurun_out/final_r152.log
done
