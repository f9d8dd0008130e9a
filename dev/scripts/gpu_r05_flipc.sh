# native per-class flip (strided dgrad-as-forward sub-filters): tests + a step A/B vs the previous commit's form is not
# switchable; the kernel trace shows the ATen flip / copy / cat kernels gone
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_conv_route_gpu.py -k "flip or strided or dgrad or graph" > gpurun_out/fc_tests.log 2>&1
: > gpurun_out/fc_ab.log
for i in 1 2; do timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o '"value": [0-9.]*' >> gpurun_out/fc_ab.log; done
( cd /tmp && export TMPDIR=/tmp && TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fc -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_fc.log 2>&1 )
