#!/bin/bash
# Round 2 (r2z): the fp64 F2 Burgers flux in the product build: full GPU
# parity suite, smoke, the bench line, and every config with config_bench's
# 0.25 s warm-up (earlier runs gave each config 3 launches, which left short
# configs measured while the clocks were still ramping).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "configs:500:python tools/config_bench.py cfg2@128 cfg4 cfg4visc cfg4cfl cfg4full cfg5 ts6 ts36 l96x1@256 l96x64@256 l96x1024@64 > gpurun_out/configs.jsonl"
