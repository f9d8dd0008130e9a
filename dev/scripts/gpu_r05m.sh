bash scripts/gpu_run.sh \
 "s_on:300:TDL_WGRAD_STREAM=0 python bench.py" \
 "s_off:300:TDL_WGRAD_STREAM=0 TDL_ROUTE_OFF=dgrad.asfwd.strided,dgrad.asfwd.strided.n64 python bench.py" \
 "s_on2:300:TDL_WGRAD_STREAM=0 python bench.py" \
 "s_off2:300:TDL_WGRAD_STREAM=0 TDL_ROUTE_OFF=dgrad.asfwd.strided,dgrad.asfwd.strided.n64 python bench.py"
