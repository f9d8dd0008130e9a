# Halo weight-gradient x-halo swizzle s&7 (in-tree build) vs (s>>1)&7 (dev/hwz0 build): exactness,
# per-kernel timing and ResNet-50 same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
OLD=$R/dev/hwz0/_C.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py tests/test_kernels_gpu.py -k "wgrad or every_route" > gpurun_out/r06_hwz.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/r06_hwz.log
for v in new old; do
[ $v = old ] && export TDL_EXT_SO=$OLD || unset TDL_EXT_SO
timeout -k 10 200 python dev/tools/dgrad_rows.py --op wgrad --shape 1024,14,256,256,3,1,1 --rows wgrad.halo.wide3x3 --rounds 3 --iters 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /"
timeout -k 10 200 python dev/tools/dgrad_rows.py --op wgrad --shape 1024,28,128,128,3,1,1 --rows wgrad.halo.wide3x3 --rounds 3 --iters 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /"
timeout -k 10 200 python dev/tools/dgrad_rows.py --op wgrad --shape 1024,7,512,512,3,1,1 --rows wgrad.halo.wide3x3 --rounds 3 --iters 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /"
done
for v in new old new old; do
[ $v = old ] && export TDL_EXT_SO=$OLD || unset TDL_EXT_SO
timeout -k 10 300 python bench.py --steps 30 > gpurun_out/r06_hwz_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_hwz_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('swz $v bench', d['value'], d['ms_per_step'])"
done
