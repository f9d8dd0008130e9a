# Interleaved A/B (5 rounds, min): default row vs the register-staged GEMM at ResNet-50 b1024 1x1 shapes
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
: > gpurun_out/r06_rsweep.log
run() { echo "## $1 $2" >> gpurun_out/r06_rsweep.log; timeout -k 10 150 python dev/tools/dgrad_rows.py --op $1 --shape $2 $3 --iters 5 --rounds 5 --rows $4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06_rsweep.log || exit 1; }
D=dgrad.asfwd.glds.n64,dgrad.asfwd.glds,dgrad.glds.stats,dgrad.glds.n64.stats,dgrad.gemm
for s in 1024,56,64,256,1,1,0 1024,56,256,64,1,1,0 1024,56,64,64,1,1,0 1024,56,256,128,1,1,0 1024,28,128,512,1,1,0 1024,28,512,128,1,1,0 1024,14,256,1024,1,1,0 1024,14,1024,256,1,1,0; do
run dgrad $s --stats $D
run wgrad $s "" wgrad.glds.1x1,wgrad.gemm
done
echo done
