#!/bin/bash
# Round 2 (r2q): linear speculative sweep with the draws computed ahead into
# LDS: small-kernel parity (bit-exact vs oracle) and config 1 end to end.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_small:300:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'small or linear or Linear or speculative or dense or fuzz or sampler'" \
  "cfg1:300:python tools/probes/cfg1_e2e.py 1 > gpurun_out/cfg1_e2e.jsonl" \
  "stuart:300:python examples/stuart_examples.py 4096 > gpurun_out/example_stuart.jsonl"
