# maxpool backward + BN sums specialised for 3x3/2 with 32-bit index math: tests, then a serial
# kernel trace of the ResNet-50 step with and without (TDL_POOL_SPEC=0) and a same-box step A/B
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "maxpool or pool" > gpurun_out/pool_tests.log 2>&1
: > gpurun_out/pool_ab.log
run() { env "$@" timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o '"value": [0-9.]*' | sed "s/^/$* /" >> gpurun_out/pool_ab.log; }
run X=spec; run TDL_POOL_SPEC=0; run X=spec; run TDL_POOL_SPEC=0
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  TDL_POOL_SPEC=$v TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_pool$v -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_pool$v.log 2>&1
done
