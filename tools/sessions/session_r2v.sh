#!/bin/bash
# Round 2 (r2v): Lorenz-96 translation units split by arithmetic mode (build
# in parallel): parity suite on the split build, and an A/B of the headline
# layouts against the pre-split build (variants/presplit) in one call.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
PRE=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/presplit/libipmc.so
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "ab_split:200:python tools/lanes_scan.py 65536 40 2000" \
  "ab_pre:200:$PRE python tools/lanes_scan.py 65536 40 2000" \
  "ab_split2:200:python tools/lanes_scan.py 65536 40 2000" \
  "ab_pre2:200:$PRE python tools/lanes_scan.py 65536 40 2000" \
  "bench:300:python bench.py > gpurun_out/bench_line.json"
