bash scripts/gpu_run.sh \
 "b_def:300:python bench.py" \
 "b_s0_256:300:TDL_WGRAD_STREAM=0 TDL_GLDS_WGRAD_TARGET=256 python bench.py" \
 "b_s0_512:300:TDL_WGRAD_STREAM=0 TDL_GLDS_WGRAD_TARGET=512 python bench.py" \
 "b_s0_1024:300:TDL_WGRAD_STREAM=0 TDL_GLDS_WGRAD_TARGET=1024 python bench.py" \
 "b_def2:300:python bench.py"
