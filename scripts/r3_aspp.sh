# round 3: GPU suite, DeepLab ASPP-join A/B, bf16 preset trace, fp32 preset PMC (MFMA busy per kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest.log 2>&1; echo "pytest rc=$?"
tail -2 gpurun_out/pytest.log
for v in 1 0 1 0; do
  TDL_ASPP_JOIN=$v timeout -k 10 300 python bench.py --model deeplab_ref --steps 40 --warmup 5 > gpurun_out/dl_$v.log 2>&1 || exit $?
  echo "aspp join=$v $(tail -1 gpurun_out/dl_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dl -o run -- \
  python3 $R/bench.py --model deeplab_ref --steps 5 --warmup 3 > $R/gpurun_out/prof_dl.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv \
  -d $R/gpurun_out/pmc_dlf32 -o run -- python3 $R/bench.py --model deeplab_ref --dtype fp32 --steps 2 --warmup 1 \
  > $R/gpurun_out/pmc_dlf32.log 2>&1 || exit $?
cd $R
python3 tools/prof_summary.py gpurun_out/prof_dl/run_kernel_trace.csv --steps 5 --marker adam_kernel --top 200 > gpurun_out/prof_dl_summary.txt 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_dlf32 --marker adam_kernel > gpurun_out/pmc_dlf32_summary.txt 2>&1
echo done
