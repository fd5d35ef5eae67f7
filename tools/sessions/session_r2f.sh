#!/bin/bash
# Round 2: in-place RK4 stages in the Lorenz-96 forward map (one array fewer
# live; same operations, so every parity test must stay bit-exact), the
# stuart_examples test, and the headline layouts at 2 / 4 waves per SIMD.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "scan_prod:300:python tools/lanes_scan.py 65536 40 2000" \
  "scan_w2:300:IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/w2/libipmc.so python tools/lanes_scan.py 65536 40 2000" \
  "scan_w4:300:IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/w4/libipmc.so python tools/lanes_scan.py 65536 40 2000" \
  "bench:300:python bench.py --no-cpu > gpurun_out/bench_line.json"
