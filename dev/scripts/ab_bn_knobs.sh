# BN elementwise launch knobs on the ResNet-50 b1024 step (same box): grid cap and backward unroll
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/bnk_ab.log
run() { env "$@" timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed "s/^/$* /" >> gpurun_out/bnk_ab.log; }
run X=default
run TDL_BN_EW_BLOCKS=2048
run TDL_BN_EW_BLOCKS=512
run TDL_BN_BWD_U=4
run X=default
run TDL_BN_EW_BLOCKS=2048
