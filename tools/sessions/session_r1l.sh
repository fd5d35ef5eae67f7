#!/bin/bash
# Full GPU suite incl. full-size parity (configs 4 and 5), torch ops, two-rank sharding.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf --durations=15"
