cd $GRAFT_REPO_ROOT
S="1024,14,256,256,3,1,1;1024,28,128,128,3,1,1;1024,7,512,512,3,1,1;1024,56,64,64,3,1,1;1024,14,1024,256,1,1,0;1024,14,256,1024,1,1,0"
for il in 0 1; do
for op in fwd dgrad; do
TDL_GLDS_IL=$il timeout -k 10 300 python3 -u tools/cfg_ab.py --op $op --shapes "$S" --cfgs 0,2,3,6 --rounds 2 > gpurun_out/cfg_${op}_$il.log 2>&1 || exit $?
done
done
