R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py -k "wgrad" tests/test_kernels_gpu.py -k "halo or wgrad" > gpurun_out/r06_h.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_h.log | tail -5
timeout -k 10 200 python dev/tools/wgrad3_ab.py 1024 > gpurun_out/r06_wgrad3_burst.txt 2>&1 || exit $?
TDL_HALO_WG_BURST=0 timeout -k 10 200 python dev/tools/wgrad3_ab.py 1024 > gpurun_out/r06_wgrad3_old.txt 2>&1 || exit $?
paste <(grep halo gpurun_out/r06_wgrad3_burst.txt) <(grep halo gpurun_out/r06_wgrad3_old.txt | awk '{print $6, $7}')
for v in 1 0 1 0; do
TDL_HALO_WG_BURST=$v timeout -k 10 300 python bench.py > gpurun_out/r06_h_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_h_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('burst $v bench', d['value'], d['ms_per_step'])"
done
bash dev/scripts/prof_r05g.sh || exit $?
head -30 gpurun_out/prof_g_summary.txt
