#!/bin/bash
# Round 2 (r2ag): Burgers CFL-mode group max by DPP + ds_swizzle instead of
# five ds_bpermute levels: Burgers parity tests, config 4 CFL A/B against the
# previous commit (variants/cflprev) twice, and the reference's Burgers study
# (CFL stepping, 1 024 chains) on both.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B=IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/cflprev/libipmc.so
C="cfg4cfl cfg4cfl:64 cfg4cfl:16 cfg4"
tools/gpu_session.sh \
  "pytest_bur:600:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'burgers or Burgers or bur'" \
  "cfl_1:300:python tools/config_bench.py $C > gpurun_out/cfl_1.jsonl" \
  "cflprev_1:300:$B python tools/config_bench.py $C > gpurun_out/cflprev_1.jsonl" \
  "cfl_2:300:python tools/config_bench.py $C > gpurun_out/cfl_2.jsonl" \
  "cflprev_2:300:$B python tools/config_bench.py $C > gpurun_out/cflprev_2.jsonl" \
  "bbeta:400:python examples/burgers_beta.py 1024 > gpurun_out/bbeta.jsonl" \
  "bbeta_prev:400:$B python examples/burgers_beta.py 1024 > gpurun_out/bbeta_prev.jsonl"
