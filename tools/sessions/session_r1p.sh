#!/bin/bash
# Burgers: fixed-dt and CFL time loops split (uniform trip count in fixed mode): parity, configs.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf" \
  "cfg_bur:300:python tools/config_bench.py cfg4 cfg4full cfg4cfl cfg4visc > gpurun_out/configs_bur_p.jsonl"
