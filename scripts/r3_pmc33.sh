# counters of one compute-bound 3x3 conv (ResNet-50 layer3 14x14x256, b1024) for each K-loop
# variant (TDL_GLDS_IL 0 / 1): fwd and dgrad
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=${1:-1024,14,256,256,3,1,1}
for il in 0 1; do
for op in fwd dgrad; do
  TDL_GLDS_IL=$il timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/p33_a_${op}_$il -o run -- python3 $R/tools/conv_one.py --op $op --shape $S --iters 5 > $R/gpurun_out/p33_a_${op}_$il.log 2>&1 || exit $?
  TDL_GLDS_IL=$il timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/p33_b_${op}_$il -o run -- python3 $R/tools/conv_one.py --op $op --shape $S --iters 5 > $R/gpurun_out/p33_b_${op}_$il.log 2>&1 || exit $?
done
done
