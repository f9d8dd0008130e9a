# dgrad-as-forward statistics + join (8-wave tiles): forced-row oracle test, then same-box A/Bs:
# (TDL_COMPUTE_PRIORITY was a temporary bench.py knob, removed after this A/B: no gain)
# TDL_BNSTAT_FUSE=1 (statistics fused into the join's last dgrad) vs the default 2, and the compute
# stream at a higher HIP priority than the weight-gradient side stream
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_route_gpu.py tests/test_kernels_gpu.py -k "route or dgrad" > gpurun_out/sj_tests.log 2>&1
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" > gpurun_out/sj_ab.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | sed 's/^/default /' >> gpurun_out/sj_ab.log
  TDL_BNSTAT_FUSE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | sed 's/^/fuse1 /' >> gpurun_out/sj_ab.log
  TDL_COMPUTE_PRIORITY=-1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | sed 's/^/prio /' >> gpurun_out/sj_ab.log
done
