# stride-2 depthwise halo de-interleave: numerics, micro timings, LDS-conflict counters
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "depthwise" tests/test_dwfold.py > gpurun_out/dws2_tests.log 2>&1
timeout -k 10 120 python dev/tools/dw_micro.py > gpurun_out/dws2_micro.log 2>&1
bash dev/scripts/pmc_dw_r05.sh
