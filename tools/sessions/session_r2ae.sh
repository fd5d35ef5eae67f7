#!/bin/bash
# Round 2 (r2ae): fp32 two-scale Lorenz-96 with the fast blocks as f32x2 pairs
# (ts_stage_pk): two-scale parity tests, then A/B against the previous commit
# (variants/tsprev), twice, warm clocks.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/tsprev/libipmc.so
C="ts6 ts36"
tools/gpu_session.sh \
  "pytest_ts:600:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'ts or two or l96ts or lorenz or thesis or run'" \
  "ts_1:300:python tools/config_bench.py $C > gpurun_out/ts_1.jsonl" \
  "tsprev_1:300:$B python tools/config_bench.py $C > gpurun_out/tsprev_1.jsonl" \
  "ts_2:300:python tools/config_bench.py $C > gpurun_out/ts_2.jsonl" \
  "tsprev_2:300:$B python tools/config_bench.py $C > gpurun_out/tsprev_2.jsonl"
