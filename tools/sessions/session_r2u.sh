#!/bin/bash
# Round 2 (r2u): in-launch samples with the speculative sweeps' incremental
# sample clock: parity suite, config 1 end to end, the reference studies
# (sample interval 1), bench line, d=40 layouts, configs.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "cfg1:300:python tools/probes/cfg1_e2e.py 1 > gpurun_out/cfg1_e2e.jsonl" \
  "lorenz_thesis:300:python examples/lorenz_thesis.py 1024 > gpurun_out/example_lorenz_thesis.json" \
  "burgers_beta:400:python examples/burgers_beta.py 1024 > gpurun_out/example_burgers_beta.jsonl" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "scan40_65k:200:python tools/lanes_scan.py 65536 40 2000" \
  "configs:500:python tools/config_bench.py cfg2@128 cfg4 cfg4visc cfg5 ts6 l96x1@256 l96x1024@64 > gpurun_out/configs.jsonl"
