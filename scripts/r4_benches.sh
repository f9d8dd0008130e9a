#!/bin/bash
# same-box benches: halo on/off, batch size, the Model loop with/without its HIP graph
bash scripts/gpu_run.sh \
  "b_halo_on:200:python -u bench.py" \
  "b_halo_off:200:TDL_HALO=0 python -u bench.py" \
  "b_1536:200:python -u bench.py --batch 1536" \
  "b_2048:240:python -u bench.py --batch 2048" \
  "b_halo_on2:200:python -u bench.py" \
  "model_loop:400:python -u bench/model_loop.py --batch 32 --steps 120 --out gpurun_out/model_loop.json" \
  "b_dl32g:200:python -u bench.py --model deeplab_ref --batch 32 --graph" \
  "b_xc2:200:python -u bench.py --model xception41 --batch 128"
