#!/bin/bash
# Round 2 (r2p): full validation at HEAD -- parity suite, smoke, bench line
# (the driver's default command), configs.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "configs:500:python tools/config_bench.py cfg2@128 cfg4 cfg4visc cfg4full cfg5 ts6 ts36 l96x1@256 l96x64@256 l96x1024@64 > gpurun_out/configs.jsonl"
