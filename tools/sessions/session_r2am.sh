#!/bin/bash
# Round 2 (r2am): small-model speculation block size (small_spec_kernel,
# IPMC_SPEC_BLOCK 256 = product vs 64 / 128 variants): the small-model parity
# tests on both variants, then config 2 A/B twice.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
V=ip_mcmc_amd/lib/variants
C="cfg2@128 cfg2@128~8 cfg2@128~32"
T="python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k small_speculative"
tools/gpu_session.sh \
  "pytest_b64:300:IPMC_LIB_PATH=$V/blk64/libipmc.so $T" \
  "pytest_b128:300:IPMC_LIB_PATH=$V/blk128/libipmc.so $T" \
  "b256_1:300:python tools/config_bench.py $C > gpurun_out/b256_1.jsonl" \
  "b64_1:300:IPMC_LIB_PATH=$V/blk64/libipmc.so python tools/config_bench.py $C > gpurun_out/b64_1.jsonl" \
  "b128_1:300:IPMC_LIB_PATH=$V/blk128/libipmc.so python tools/config_bench.py $C > gpurun_out/b128_1.jsonl" \
  "b256_2:300:python tools/config_bench.py $C > gpurun_out/b256_2.jsonl" \
  "b64_2:300:IPMC_LIB_PATH=$V/blk64/libipmc.so python tools/config_bench.py $C > gpurun_out/b64_2.jsonl" \
  "b128_2:300:IPMC_LIB_PATH=$V/blk128/libipmc.so python tools/config_bench.py $C > gpurun_out/b128_2.jsonl"
