#!/bin/bash
# torch.ops front end after the ABI 7 rebuild; two-scale K=6 with two slow
# variables per lane (3 lanes per chain) vs the default 6.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_torch:200:python -u -m pytest tests/test_torch_ops.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "ts6_spl2:300:python tools/config_bench.py ts6 ts6:3 > gpurun_out/ts6_spl.jsonl"
