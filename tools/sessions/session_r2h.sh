#!/bin/bash
# A/B on one box: the in-place RK4 stage (product) vs the previous header
# (variants/old: rates array, 6 live arrays) for d=40 / d=36 layouts and cfg 5.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
OLD=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/old/libipmc.so
tools/gpu_session.sh \
  "ab_new40:200:python tools/lanes_scan.py 65536 40 2000" \
  "ab_old40:200:$OLD python tools/lanes_scan.py 65536 40 2000" \
  "ab_new36:200:python tools/lanes_scan.py 65536 36 2000" \
  "ab_old36:200:$OLD python tools/lanes_scan.py 65536 36 2000" \
  "ab_new_cfg5:200:python tools/config_bench.py cfg5 > gpurun_out/ab_new_cfg5.jsonl" \
  "ab_old_cfg5:200:$OLD python tools/config_bench.py cfg5 > gpurun_out/ab_old_cfg5.jsonl" \
  "ab_new_cfg5b:200:python tools/config_bench.py cfg5 > gpurun_out/ab_new_cfg5b.jsonl"
