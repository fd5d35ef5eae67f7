#!/bin/bash
# Re-entry check: full GPU parity suite, smoke, the bench line and the Burgers configs.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "cfg_bur:300:python tools/config_bench.py cfg4 cfg4full cfg4cfl cfg4visc > gpurun_out/configs_bur.jsonl"
