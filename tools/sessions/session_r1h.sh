#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_diag:600:python -m pytest tests/test_gpu_diag.py -q -p no:cacheprovider --timeout 500 -rf" \
  "cfg_ts:300:python tools/config_bench.py ts6 ts36"
