# where does the memory-free (TDL_CONV_DBG=192: no DMA, no epilogue loads/stores) 1x1 dgrad spend
# its cycles? instruction mix and stall counters, full kernel vs memory-free
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=256,56,256,64,1,1,0
for dbg in 0 192; do
  TDL_CONV_DBG=$dbg timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcd2_a_$dbg -o run -- python3 $R/tools/conv_one.py --op dgrad --shape $S --iters 5 > $R/gpurun_out/pmcd2_a_$dbg.log 2>&1 || exit $?
  TDL_CONV_DBG=$dbg timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcd2_b_$dbg -o run -- python3 $R/tools/conv_one.py --op dgrad --shape $S --iters 5 > $R/gpurun_out/pmcd2_b_$dbg.log 2>&1 || exit $?
done
