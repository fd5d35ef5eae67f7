#!/bin/bash
# Round 2 (r2t): ABI 9 -- samples recorded inside a launch (sample_every):
# the run-vs-per-sample tests over every kernel family, the full parity suite,
# the reference studies with sample interval 1 (examples), config 1.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_run:400:python -u -m pytest tests/test_gpu_run.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "cfg1:300:python tools/probes/cfg1_e2e.py 1 > gpurun_out/cfg1_e2e.jsonl" \
  "lorenz_thesis:300:python examples/lorenz_thesis.py 1024 > gpurun_out/example_lorenz_thesis.json" \
  "burgers_beta:400:python examples/burgers_beta.py 1024 > gpurun_out/example_burgers_beta.jsonl" \
  "bench:300:python bench.py --no-cpu > gpurun_out/bench_line.json"
