bash scripts/gpu_run.sh \
 "route_r50:300:python tools/route_report.py --model resnet50 --batch 1024" \
 "route_x41:300:python tools/route_report.py --model xception_41 --batch 64 --image 299" \
 "t_route:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_route_gpu.py -p no:cacheprovider"
