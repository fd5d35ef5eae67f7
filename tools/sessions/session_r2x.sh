#!/bin/bash
# Round 2 (r2x): the fp64 F2 Burgers flux as the product path: Burgers parity
# tests, then config 4 at 8 and 4 cells per lane (0.25 s warm-up per config).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_bur:600:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'burgers or Burgers or bur'" \
  "cfg_bur_a:300:python tools/config_bench.py cfg4 cfg4:64 cfg4visc cfg4visc:64 cfg4cfl cfg4cfl:64 cfg4full cfg4full:64 > gpurun_out/cfg_bur_a.jsonl" \
  "cfg_bur_b:300:python tools/config_bench.py cfg4:64 cfg4 cfg4visc:64 cfg4visc cfg4cfl:64 cfg4cfl cfg4full:64 cfg4full > gpurun_out/cfg_bur_b.jsonl"
