# In-step A/B of scheduling knobs on the final build (ResNet-50 b1024, 30 steps, alternating)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
b() { env "$@" timeout -k 10 300 python bench.py --steps 30 > gpurun_out/r06_knobs_bench.log 2>&1 || exit 1
      tail -1 gpurun_out/r06_knobs_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do
b TDL_NONE=1
b TDL_GLDS_WGRAD_TARGET=96
b TDL_GLDS_WGRAD_TARGET=160
b TDL_HALO_WG_TARGET=384
b TDL_WGRAD_EARLY=0
b TDL_ROUTE_ON=fwd.glds.stem
done
