# Experimental switches re-checked on the final build (ResNet-50 b1024, 30 steps, alternating)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
b() { env "$@" timeout -k 10 300 python bench.py --steps 30 > gpurun_out/r06_exp_bench.log 2>&1 || exit 1
      tail -1 gpurun_out/r06_exp_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'])"; }
for rep in 1 2; do
b TDL_NONE=1
b TDL_EXPERIMENTAL=m32
b TDL_EXPERIMENTAL=join_stats
b TDL_EXPERIMENTAL=stem_glds
done
