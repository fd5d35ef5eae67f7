#!/bin/bash
# New Lorenz-96 layout rule: whole GPU suite (layouts change for many ensemble sizes), then the auto picks timed.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "suite:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider" \
  "auto:400:for c in 8192 16384 32768 65536; do python tools/config_bench.py l96x\$c 2>/dev/null || exit 1; done > gpurun_out/auto_layouts.jsonl"
