#!/bin/bash
# Round 2 (r2aj): Lorenz-63 speculation with two slots per lane (fp32 as
# v_pk_* pairs; fp64 pairs as a variant): the small-model and run() parity
# tests on the product and on the fp64-pair variant, then config 2 A/B
# against the one-slot kernel (variants/l63base) twice, 128 pCN steps per
# launch (a first call ran one step per launch: round cost only).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
V=ip_mcmc_amd/lib/variants
C="cfg2@128 cfg2@128~16 cfg2@128~32 cfg2@128~64"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_run.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf"
tools/gpu_session.sh \
  "pytest_l63:600:$T -k 'small or l63 or Lorenz63 or pcn_run or overlapped'" \
  "pytest_pair64:600:IPMC_LIB_PATH=$V/l63pair64/libipmc.so $T -k 'small or l63 or Lorenz63'" \
  "new_1:300:python tools/config_bench.py $C > gpurun_out/new_1.jsonl" \
  "base_1:300:IPMC_LIB_PATH=$V/l63base/libipmc.so python tools/config_bench.py $C > gpurun_out/base_1.jsonl" \
  "pair64_1:300:IPMC_LIB_PATH=$V/l63pair64/libipmc.so python tools/config_bench.py $C > gpurun_out/pair64_1.jsonl" \
  "new_2:300:python tools/config_bench.py $C > gpurun_out/new_2.jsonl" \
  "base_2:300:IPMC_LIB_PATH=$V/l63base/libipmc.so python tools/config_bench.py $C > gpurun_out/base_2.jsonl" \
  "pair64_2:300:IPMC_LIB_PATH=$V/l63pair64/libipmc.so python tools/config_bench.py $C > gpurun_out/pair64_2.jsonl"
