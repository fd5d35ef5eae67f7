#!/bin/bash
# Two-scale Lorenz-96 occupancy scan: the product build (4 waves/SIMD for K=6
# J=4 f64) vs launch bounds for 5 / 6 / 8 waves (variants/ts_w*).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "ts_base:200:python tools/config_bench.py ts6 ts36 > gpurun_out/ts_base.jsonl" \
  "ts_w5:200:IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/ts_w5/libipmc.so python tools/config_bench.py ts6 ts36 > gpurun_out/ts_w5.jsonl" \
  "ts_w6:200:IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/ts_w6/libipmc.so python tools/config_bench.py ts6 ts36 > gpurun_out/ts_w6.jsonl" \
  "ts_w8:200:IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/ts_w8/libipmc.so python tools/config_bench.py ts6 ts36 > gpurun_out/ts_w8.jsonl"
