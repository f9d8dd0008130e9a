# depthwise kernel counters (dev/tools/dw_micro.py), one pass per counter group
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 $R/tools/dw_micro.py > $R/gpurun_out/dw_micro.log 2>&1 || exit $?
p() { tag=$1; shift; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/pmcdw_$tag -o run -- python3 $R/tools/dw_micro.py > $R/gpurun_out/pmcdw_$tag.log 2>&1; }
p sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit $?
p fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
p ta TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit $?
