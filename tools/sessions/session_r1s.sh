#!/bin/bash
# Config table refresh on the current build.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "configs:500:python tools/config_bench.py cfg2 cfg2@128 cfg4 cfg4full cfg4cfl cfg4visc cfg5 ts6 ts36 l96x1@64 l96x64@64 l96x1024@64 > gpurun_out/configs_s.jsonl"
