#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:1500:python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 900 -rf -x" \
  "lanes40:600:python tools/lanes_scan.py 65536 40 2000" \
  "lanes256:900:python tools/lanes_scan.py 131072 256 2000" \
  "bench:900:python bench.py --steps 20 --warmup 3"
