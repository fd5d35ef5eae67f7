#!/bin/bash
# Round 2 (r2aa): fp32 Burgers on cell pairs (rus_rate_pk, v_pk_* F2 flux):
# Burgers parity tests, then A/B against the previous commit's fp32 flux
# (variants/burprev), twice, warm clocks.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/burprev/libipmc.so
C="cfg4 cfg4visc cfg4cfl cfg4full cfg4:64"
tools/gpu_session.sh \
  "pytest_bur:600:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'burgers or Burgers or bur'" \
  "pk_1:300:python tools/config_bench.py $C > gpurun_out/pk_1.jsonl" \
  "prev_1:300:$B python tools/config_bench.py $C > gpurun_out/prev_1.jsonl" \
  "pk_2:300:python tools/config_bench.py $C > gpurun_out/pk_2.jsonl" \
  "prev_2:300:$B python tools/config_bench.py $C > gpurun_out/prev_2.jsonl"
