# round 3: 256x256 forward tiles (cfg 8, 2-stage ring) vs the default 256x128 (cfg 0); fp32 preset bench; dadd kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "join_dadd or m32" --timeout 200 --timeout-method thread > gpurun_out/pytest_dadd.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_dadd.log
timeout -k 10 300 python tools/cfg_ab.py --op fwd --cfgs 0,8 --rounds 3 \
  --shapes "1024,14,256,256,3,1,1;1024,28,128,128,3,1,1;1024,7,512,512,3,1,1;1024,14,1024,256,1,1,0;1024,14,256,1024,1,1,0;1024,28,128,512,1,1,0" \
  > gpurun_out/cfg8.log 2>&1 || exit $?
cat gpurun_out/cfg8.log
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --steps 30 --warmup 5 > gpurun_out/dlf32_slab.log 2>&1 || exit $?
tail -1 gpurun_out/dlf32_slab.log
echo done
