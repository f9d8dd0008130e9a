# Every route row forced at the Xception-41 b128 conv shapes (fwd / dgrad with BN sums, wgrad)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
: > gpurun_out/r06_xsweep.log
for shp in 128,150,64,128,1,1,0 128,150,128,128,1,1,0 128,75,128,256,1,1,0 128,75,256,256,1,1,0 128,75,128,128,1,1,0 128,38,256,728,1,1,0 128,38,728,728,1,1,0 128,19,728,728,1,1,0 128,19,728,1024,1,1,0 128,10,1024,1536,1,1,0 128,10,1536,1536,1,1,0 128,10,1536,2048,1,1,0 128,150,64,128,1,2,0 128,75,128,256,1,2,0 128,38,256,728,1,2,0 128,19,728,1024,1,2,0 128,150,32,64,3,1,1 128,299,8,32,3,2,1; do
for op in fwd dgrad wgrad; do
st=--stats; [ $op = wgrad ] && st=
echo "## $op $shp" >> gpurun_out/r06_xsweep.log
timeout -k 10 120 python dev/tools/dgrad_rows.py --op $op --shape $shp $st --iters 5 2>&1 | grep -v amdgpu.ids | grep -v " -  (" >> gpurun_out/r06_xsweep.log || exit 1
done; done
echo done
