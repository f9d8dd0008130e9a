# fp8 route-row tile configs on the ResNet-152 b256 fp8 graph step, same box
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/f8cfg_ab.log
run() { env "$@" timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed "s/^/$* /" >> gpurun_out/f8cfg_ab.log; }
run X=default
run TDL_ROUTE_CFG=dgrad.glds.fp8:1
run TDL_ROUTE_CFG=wgrad.glds.fp8:2
run TDL_ROUTE_CFG=fwd.glds.fp8:1
run X=default
