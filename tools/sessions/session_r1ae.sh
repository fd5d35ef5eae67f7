#!/bin/bash
# Two-scale K=6 J=4 f64 occupancy: 4 waves/SIMD (default, 1.6 rounds of waves) vs 6 and 7 (one round, some scratch spills).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "ts_w4:300:python tools/config_bench.py ts6 > gpurun_out/ts_w4.jsonl" \
  "ts_w6:300:IPMC_LIB_PATH=\$PWD/ip_mcmc_amd/lib_w6/libipmc.so python tools/config_bench.py ts6 > gpurun_out/ts_w6.jsonl" \
  "ts_w7:300:IPMC_LIB_PATH=\$PWD/ip_mcmc_amd/lib_w7/libipmc.so python tools/config_bench.py ts6 > gpurun_out/ts_w7.jsonl"
