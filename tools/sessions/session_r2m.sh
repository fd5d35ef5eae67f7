#!/bin/bash
# Round 2 (r2m): viscous Burgers with the viscous flux folded into the Rusanov
# wave-speed term (FMA arith): parity (GPU vs oracle, bit-exact), cfg 4
# timings (inviscid / viscous / CFL), the stuart_examples script, bench line.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_burgers:400:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'burgers or Burgers'" \
  "configs:400:python tools/config_bench.py cfg4 cfg4visc cfg4cfl cfg4full > gpurun_out/configs_burgers.jsonl" \
  "stuart:300:python examples/stuart_examples.py 4096 > gpurun_out/example_stuart.jsonl" \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "bench:300:python bench.py > gpurun_out/bench_line.json"
