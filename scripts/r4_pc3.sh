#!/bin/bash
# PC auto-route + fold without the dy column sums: numerics, whole-step A/Bs, Xception profile
bash scripts/gpu_run.sh \
  "tests:400:python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_bnfold.py tests/test_serving.py tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -k 'fold or serving or export or xception or producer_consumer or resnet'" \
  "r50_auto:200:python -u bench.py" \
  "r50_pc0:200:TDL_CONV_PC=0 python -u bench.py" \
  "r50_auto_b:200:python -u bench.py" \
  "r50_pc0_b:200:TDL_CONV_PC=0 python -u bench.py" \
  "xc_fold:200:python -u bench.py --model xception41 --batch 128" \
  "xc_nofold:200:TDL_BN_CONV_FOLD=0 python -u bench.py --model xception41 --batch 128" \
  "xc_fold_b:200:python -u bench.py --model xception41 --batch 128" \
  "xc_nofold_b:200:TDL_BN_CONV_FOLD=0 python -u bench.py --model xception41 --batch 128" \
  "prof_xc3:300:bash scripts/prof_bench.sh xc3 --model xception41 --batch 128" \
  "model_loop:500:python -u bench/model_loop.py --batch 32 --steps 120 --modes auto:4:20,auto:4:0,auto:12:0,auto:12:20 --out gpurun_out/model_loop2.json"
