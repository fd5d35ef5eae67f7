#!/bin/bash
# Round 2 (r2y): clean A/B (0.25 s warm-up per config) of the fp64 F2 Burgers
# flux (product) against the previous flux form (variants/burbase), twice.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/burbase/libipmc.so
C="cfg4 cfg4visc cfg4cfl cfg4full"
tools/gpu_session.sh \
  "f2_1:300:python tools/config_bench.py $C > gpurun_out/f2_1.jsonl" \
  "base_1:300:$B python tools/config_bench.py $C > gpurun_out/base_1.jsonl" \
  "f2_2:300:python tools/config_bench.py $C > gpurun_out/f2_2.jsonl" \
  "base_2:300:$B python tools/config_bench.py $C > gpurun_out/base_2.jsonl"
