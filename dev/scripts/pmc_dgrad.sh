# hardware counters of the LDS-DMA 1x1 dgrad (ResNet-50 layer1 join shape), full vs epilogue-free
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=256,56,256,64,1,1,0
for dbg in 0 128; do
  TDL_CONV_DBG=$dbg timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcdg_sq_$dbg -o run -- python3 $R/tools/conv_one.py --op dgrad --shape $S --iters 5 > $R/gpurun_out/pmcdg_sq_$dbg.log 2>&1 || exit $?
  TDL_CONV_DBG=$dbg timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TA_BUFFER_READ_LDS_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcdg_ta_$dbg -o run -- python3 $R/tools/conv_one.py --op dgrad --shape $S --iters 5 > $R/gpurun_out/pmcdg_ta_$dbg.log 2>&1 || exit $?
  TDL_CONV_DBG=$dbg timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcdg_mem_$dbg -o run -- python3 $R/tools/conv_one.py --op dgrad --shape $S --iters 5 > $R/gpurun_out/pmcdg_mem_$dbg.log 2>&1 || exit $?
done
