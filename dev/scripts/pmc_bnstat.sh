# hardware counters: BN-backward statistics fused into the dgrad epilogue vs dgrad + BN reduce
# (ResNet-50 layer2 conv3 dgrad, 28x28 512 -> 128 at b256)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=256,28,128,512,1,1,0
for op in dgrad_bnstat dgrad_reduce; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcbs_fetch_$op -o run -- python3 $R/tools/conv_one.py --op $op --shape $S --iters 5 > $R/gpurun_out/pmcbs_fetch_$op.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcbs_write_$op -o run -- python3 $R/tools/conv_one.py --op $op --shape $S --iters 5 > $R/gpurun_out/pmcbs_write_$op.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcbs_sq_$op -o run -- python3 $R/tools/conv_one.py --op $op --shape $S --iters 5 > $R/gpurun_out/pmcbs_sq_$op.log 2>&1 || exit $?
done
