#!/bin/bash
# Round 2 (r2ad): Lorenz-63 FMA step with an 8-op dependent chain (was 13):
# small-model parity tests, then config 2 A/B against the previous commit's
# ipmc_api (variants/l63prev) at speculation widths 16 / 8 / 32, twice.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/l63prev/libipmc.so
C="cfg2@128 cfg2@128:8 cfg2@128:32 cfg2"
tools/gpu_session.sh \
  "pytest_small:600:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'l63 or L63 or lorenz63 or Lorenz63 or small or spec or run or example'" \
  "l63_1:300:python tools/config_bench.py $C > gpurun_out/l63_1.jsonl" \
  "l63prev_1:300:$B python tools/config_bench.py $C > gpurun_out/l63prev_1.jsonl" \
  "l63_2:300:python tools/config_bench.py $C > gpurun_out/l63_2.jsonl" \
  "l63prev_2:300:$B python tools/config_bench.py $C > gpurun_out/l63prev_2.jsonl"
