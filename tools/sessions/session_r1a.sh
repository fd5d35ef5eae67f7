#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
tools/gpu_session.sh \
  "probe:120:./build/valu_probe" \
  "pytest_gpu:1200:python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 -rf" \
  "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:900:python bench.py --steps 20 --warmup 3"
