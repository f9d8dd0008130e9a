# wgrad.halo.3x3 (3x3 weight gradients from 64 inputs / 32k rows on the halo kernel): per-shape
# timings at b256, then a same-box step A/B against the row switched off
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
N=256 timeout -k 10 300 python dev/tools/wgrad_rows_ab.py > gpurun_out/wgrad_rows256.log 2>&1
: > gpurun_out/wh_ab.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed 's/^/on  /' >> gpurun_out/wh_ab.log
  TDL_ROUTE_OFF=wgrad.halo.3x3 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed 's/^/off /' >> gpurun_out/wh_ab.log
done
