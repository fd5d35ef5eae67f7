#!/bin/bash
# Round 2 (r2w): Burgers flux in the F2 scale (per-cell squares and wave
# speeds, 4 VALU ops per interface; variants/burf2) vs the product flux form,
# A/B twice on one box, and 4 cells per lane (64 lanes per chain) for both.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
F2=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/burf2/libipmc.so
C="cfg4 cfg4full cfg4visc cfg4cfl cfg4:64"
tools/gpu_session.sh \
  "ab_base1:300:python tools/config_bench.py $C > gpurun_out/ab_base1.jsonl" \
  "ab_f2_1:300:$F2 python tools/config_bench.py $C > gpurun_out/ab_f2_1.jsonl" \
  "ab_base2:300:python tools/config_bench.py $C > gpurun_out/ab_base2.jsonl" \
  "ab_f2_2:300:$F2 python tools/config_bench.py $C > gpurun_out/ab_f2_2.jsonl"
