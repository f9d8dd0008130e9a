# TDL_BNSTAT_FUSE 1 vs 2, longer alternating A/B (40 timed steps each)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for v in 1 2 1 2 1 2; do
TDL_BNSTAT_FUSE=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/r06_js_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_js_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bnstat_fuse $v bench', d['value'], d['ms_per_step'])"
done
