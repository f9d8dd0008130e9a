# Stem pool kernels in isolation: timing + PMC passes (one kernel family per run)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python dev/tools/pool_bench.py > gpurun_out/poolb.log 2>&1 || exit $?
cat gpurun_out/poolb.log
cd /tmp && export TMPDIR=/tmp
for what in fwd bwd copy; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_pool_${what}_a -o run -- python3 $R/dev/tools/pool_bench.py --only $what --iters 3 > /dev/null 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $R/gpurun_out/pmc_pool_${what}_b -o run -- python3 $R/dev/tools/pool_bench.py --only $what --iters 3 > /dev/null 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $R/gpurun_out/pmc_pool_${what}_c -o run -- python3 $R/dev/tools/pool_bench.py --only $what --iters 3 > /dev/null 2>&1 || exit $?
done
echo done
