#!/bin/bash
# Round 2 (r2ab): Burgers parity tests incl. fp32 layouts / viscous / ghost-edge cases.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_bur:600:python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'burgers or Burgers or bur'"
