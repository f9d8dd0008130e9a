#!/bin/bash
# stride-2 depthwise dgrad kernel: numerics + micro + Xception; serving/fp8 tests; Model-loop kernel trace
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash scripts/gpu_run.sh \
  "dw_tests:300:python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_f32_gpu.py -m gpu -k 'depthwise or xception or dw'" \
  "dw_micro:200:python -u tools/dw_micro.py" \
  "serve:300:python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_serving.py tests/test_bnfold.py -m gpu" \
  "xc:200:python -u bench.py --model xception41 --batch 128" \
  "xc_s2off:200:TDL_DW_S2_OFF=1 python -u bench.py --model xception41 --batch 128" \
  "prof_loop:400:cd /tmp && timeout -k 10 380 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_loop -o run -- python3 $R/bench/model_loop.py --batch 32 --steps 60 --modes auto:4:0"
