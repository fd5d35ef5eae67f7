#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:1500:python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 900 -rf"
