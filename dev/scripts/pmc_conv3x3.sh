# MFMA / issue / wait counters of a compute-bound 3x3 conv (ResNet-50 layer3, b256) on the
# LDS-DMA kernel: forward and dgrad
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=256,14,256,256,3,1,1
for op in fwd dgrad; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc33_a_$op -o run -- python3 $R/tools/conv_one.py --op $op --shape $S --iters 5 > $R/gpurun_out/pmc33_a_$op.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc33_b_$op -o run -- python3 $R/tools/conv_one.py --op $op --shape $S --iters 5 > $R/gpurun_out/pmc33_b_$op.log 2>&1 || exit $?
done
