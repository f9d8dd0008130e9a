# remaining stream / halo knobs on the ResNet-50 b1024 step, same box
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/misc_ab.log
run() { env "$@" timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed "s/^/$* /" >> gpurun_out/misc_ab.log; }
run X=default
run TDL_WGRAD_EARLY=0
run TDL_HALO_WG_TARGET=256
run TDL_HALO_WG_TARGET=1024
run TDL_BN_RED_BLOCKS=2048
run X=default
