#!/bin/bash
# Round 2, first GPU call: parity after the ADVICE fixes (ABI 6: chain-id and
# step ranges, ipmc_plan_sweep, long-series autocorrelation, RNG continuation
# across runs, resume checks), smoke, the bench line, and the f64 MFMA probe.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/bin
tools/gpu_session.sh \
  "pytest_gpu:700:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "mfma_build:120:/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w tools/mfma_f64_probe.hip -o gpurun_out/bin/mfma_f64_probe" \
  "mfma_probe:120:gpurun_out/bin/mfma_f64_probe > gpurun_out/mfma_f64_probe.txt"
