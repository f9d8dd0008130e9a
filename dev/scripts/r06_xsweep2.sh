# Interleaved A/B of the default row vs the register-staged GEMM at the Xception shapes where the
# one-pass sweep flagged it (5 rounds, min)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
: > gpurun_out/r06_xsweep2.log
run() { echo "## $1 $2" >> gpurun_out/r06_xsweep2.log; timeout -k 10 120 python dev/tools/dgrad_rows.py --op $1 --shape $2 $3 --iters 5 --rounds 5 --rows $4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06_xsweep2.log || exit 1; }
run dgrad 128,150,64,128,1,1,0 --stats dgrad.asfwd.glds.n64,dgrad.asfwd.glds,dgrad.gemm,dgrad.glds.stats
run dgrad 128,150,128,128,1,1,0 --stats dgrad.asfwd.glds,dgrad.gemm,dgrad.glds.stats
run dgrad 128,75,128,128,1,1,0 --stats dgrad.asfwd.glds,dgrad.gemm,dgrad.glds.stats
run dgrad 128,75,128,256,1,1,0 --stats dgrad.asfwd.glds,dgrad.gemm,dgrad.glds.stats
run dgrad 128,150,64,128,1,2,0 --stats dgrad.asfwd.strided.n64,dgrad.asfwd.strided,dgrad.gemm,dgrad.glds.stats
run wgrad 128,75,256,256,1,1,0 "" wgrad.glds.1x1,wgrad.gemm
run wgrad 128,38,256,728,1,1,0 "" wgrad.glds.1x1,wgrad.gemm
run wgrad 128,38,728,728,1,1,0 "" wgrad.glds.1x1,wgrad.gemm
run wgrad 128,38,256,728,1,2,0 "" wgrad.glds.1x1,wgrad.gemm
run fwd 128,75,128,128,1,1,0 --stats fwd.glds.wide,fwd.glds.aligned,fwd.gemm
echo done
