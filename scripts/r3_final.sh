# round 3 validation: full GPU suite, driver smoke, headline bench, model benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_all.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --model xception41 --image-size 299 --batch 128 > gpurun_out/bench_xc.log 2>&1 || exit $?
tail -1 gpurun_out/bench_xc.log
timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph > gpurun_out/bench_r152f8.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r152f8.log
timeout -k 10 300 python bench.py --model deeplab_ref --steps 40 > gpurun_out/bench_dl.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dl.log
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --steps 30 > gpurun_out/bench_dlf32.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dlf32.log
echo done
