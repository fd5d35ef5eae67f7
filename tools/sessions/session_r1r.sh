#!/bin/bash
# Burgers CFL group max via v_max; two-scale K=6 with two slow variables per lane.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_bur:600:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf -k 'burgers or Burgers or random or cfg4'" \
  "cfg:300:python tools/config_bench.py cfg4cfl ts6 ts6:3 > gpurun_out/configs_r.jsonl"
