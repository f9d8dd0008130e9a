# Xception-41 b128 in-step A/B of LDS-DMA tile configs after the grouped-tiling fix
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
b() { env "$@" timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 --steps 30 > gpurun_out/r06_xk.log 2>&1 || exit 1
      tail -1 gpurun_out/r06_xk.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do
b TDL_NONE=1
b TDL_ROUTE_CFG=fwd.glds.wide:3 TDL_GLDS_SLOTS=512
b TDL_ROUTE_CFG=fwd.glds.wide:2
b TDL_ROUTE_CFG=dgrad.glds.stats:3 TDL_GLDS_SLOTS=512
b TDL_ROUTE_CFG=dgrad.asfwd.glds:4
done
