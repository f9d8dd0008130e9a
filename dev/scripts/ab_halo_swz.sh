set -e
# (the A/B needs the temporary TDL_HALO_SWZ toggle, which is not in the tree: the result is in profiles/r05_halo_narrow_pmc.txt)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/halo_ab.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed 's/^/swz1 /' >> gpurun_out/halo_ab.log
  TDL_HALO_SWZ=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed 's/^/swz0 /' >> gpurun_out/halo_ab.log
done
