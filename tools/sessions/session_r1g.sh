#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_ts:600:python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 500 -rf -k 'l96ts or chainio'" \
  "pytest_gpu:900:python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 800 -rf"
