#!/bin/bash
# Round 2 (r2af): two-scale occupancy targets after the fp32 pair layout
# (variants/tsw5, tsw6 force 5 / 6 waves per SIMD for every instantiation;
# product: ts_waves), twice.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
W5=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/tsw5/libipmc.so
W6=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/tsw6/libipmc.so
C="ts6 ts36"
tools/gpu_session.sh \
  "tsw_p1:300:python tools/config_bench.py $C > gpurun_out/tsw_p1.jsonl" \
  "tsw_5a:300:$W5 python tools/config_bench.py $C > gpurun_out/tsw_5a.jsonl" \
  "tsw_6a:300:$W6 python tools/config_bench.py $C > gpurun_out/tsw_6a.jsonl" \
  "tsw_p2:300:python tools/config_bench.py $C > gpurun_out/tsw_p2.jsonl" \
  "tsw_5b:300:$W5 python tools/config_bench.py $C > gpurun_out/tsw_5b.jsonl" \
  "tsw_6b:300:$W6 python tools/config_bench.py $C > gpurun_out/tsw_6b.jsonl"
