# Stem pool kernel on the ResNet-50 step's own tensors vs fresh copies
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python dev/tools/pool_inbench.py > gpurun_out/pool_inbench.log 2>&1; rc=$?
cat gpurun_out/pool_inbench.log | grep -v amdgpu.ids; exit $rc
