bash scripts/gpu_run.sh \
 "bnconv_tests:600:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bnconv.py -m gpu -p no:cacheprovider" \
 "bench_fold:300:python bench.py" \
 "bench_nofold:300:TDL_BN_CONV_FOLD=0 python bench.py"
