bash scripts/gpu_run.sh \
  "gpu_suite:1000:python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider" \
  "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "dp2:300:bash scripts/rehearse_dp2.sh" \
  "bench:300:python bench.py"
