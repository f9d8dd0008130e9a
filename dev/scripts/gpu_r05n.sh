X="python bench.py --model xception41 --batch 128 --image-size 299"
bash scripts/gpu_run.sh \
 "c0:300:$X" \
 "c2:300:TDL_ROUTE_CFG=wgrad.glds.1x1:2 $X" \
 "c3:300:TDL_ROUTE_CFG=wgrad.glds.1x1:3 $X" \
 "c1:300:TDL_ROUTE_CFG=wgrad.glds.1x1:1 $X" \
 "c0t256:300:TDL_GLDS_WGRAD_TARGET=256 $X" \
 "c0b:300:$X"
