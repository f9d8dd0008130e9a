# persistent-grid size of the LDS-DMA conv kernels and the 32x32 MFMA dgrad, ResNet-50 b1024, same box
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/slots_ab.log
run() { env "$@" timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed "s/^/$* /" >> gpurun_out/slots_ab.log; }
run X=default
run TDL_GLDS_SLOTS=224
run TDL_GLDS_SLOTS=192
run TDL_GLDS_SLOTS=320
run TDL_GLDS_SLOTS=512
run TDL_M32=1
run X=default
