set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 bench/conv_bench.py --batch 1024 --out gpurun_out/conv_bench_b1024_r3base.json > gpurun_out/conv_bench_b1024_r3base.log 2>&1 || exit $?
bash scripts/prof_bench.sh r3base || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r3base/run_kernel_trace.csv --steps 5 > gpurun_out/prof_r3base_summary.txt 2>&1
