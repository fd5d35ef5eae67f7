#!/bin/bash
# Constrained-chain fixture on the device, then the whole GPU suite and smoke.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "con:180:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k constrained" \
  "suite:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider" \
  "smoke:180:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
