#!/bin/bash
# Small-ensemble layout rule (DPP halos below one wave per SIMD): GPU suite, then the auto picks timed.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "suite:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider" \
  "auto:300:python tools/config_bench.py l96x1@64 l96x64@64 l96x1024@64 > gpurun_out/l96_small_auto.jsonl"
