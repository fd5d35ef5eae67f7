#!/bin/bash
# FMA-arith folds (Burgers SSPRK2 average, two-scale 1/J and c): parity, configs, Burgers layouts.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf" \
  "cfg:400:python tools/config_bench.py cfg4 cfg4full cfg4cfl cfg4visc ts6 ts36 > gpurun_out/configs_j.jsonl" \
  "cfg_lay:300:python tools/config_bench.py cfg4:64 cfg4full:64 cfg4:32 > gpurun_out/configs_bur_lay.jsonl"
