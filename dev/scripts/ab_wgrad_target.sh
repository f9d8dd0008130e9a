# weight-gradient split-K target (TDL_GLDS_WGRAD_TARGET, default 128 workgroups), same box:
# ResNet-152 fp8 graph and ResNet-50 bf16
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/wt_ab.log
r152() { env "$@" timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed "s/^/r152fp8 $* /" >> gpurun_out/wt_ab.log; }
r50() { env "$@" timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed "s/^/r50 $* /" >> gpurun_out/wt_ab.log; }
r152 X=default
r152 TDL_GLDS_WGRAD_TARGET=64
r152 TDL_GLDS_WGRAD_TARGET=256
r152 X=default
r50 X=default
r50 TDL_GLDS_WGRAD_TARGET=64
r50 X=default
