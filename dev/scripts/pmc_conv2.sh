# cache-path counters for two representative conv shapes under both kernel implementations
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for shp in 256,56,64,64,3,1,1 256,14,512,512,3,2,1; do
 for m in 0 2; do
  tag=$(echo $shp | tr , _)_m$m
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $R/gpurun_out/pmcA_$tag -o run -- python3 $R/tools/conv_one.py --mode $m --op fwd --shape $shp --iters 3 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum --output-format csv -d $R/gpurun_out/pmcB_$tag -o run -- python3 $R/tools/conv_one.py --mode $m --op fwd --shape $shp --iters 3 || exit $?
 done
done
