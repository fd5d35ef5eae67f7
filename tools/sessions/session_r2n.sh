#!/bin/bash
# Round 2 (r2n): the native C++ caller of the C-ABI against the oracle, and
# its own timing line at the headline size.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_capi:300:python -u -m pytest tests/test_gpu_c_api.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "capi_run:120:examples/c_api/l96_pcn 65536 1 > gpurun_out/c_api_l96_pcn.jsonl && examples/c_api/l96_pcn 65536 10 >> gpurun_out/c_api_l96_pcn.jsonl"
