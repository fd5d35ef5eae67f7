#!/bin/bash
# Round 2 (r2ap): Burgers 8 vs 4 cells per lane (32 vs 64 lanes per chain) on
# the current kernels (F2 flux, fp32 cell pairs, DPP CFL max), twice.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
C="cfg4 cfg4:64 cfg4cfl cfg4cfl:64 cfg4visc cfg4visc:64 cfg4full cfg4full:64"
tools/gpu_session.sh \
  "bur_1:400:python tools/config_bench.py $C > gpurun_out/bur_1.jsonl" \
  "bur_2:400:python tools/config_bench.py $C > gpurun_out/bur_2.jsonl"
