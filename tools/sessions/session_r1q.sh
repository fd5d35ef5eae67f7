#!/bin/bash
# Burgers: max(|a|,|b|) as one v_max with abs modifiers: parity, configs.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf" \
  "cfg_bur:300:python tools/config_bench.py cfg4 cfg4full cfg4cfl cfg4visc > gpurun_out/configs_bur_q.jsonl"
