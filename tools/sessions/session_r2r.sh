#!/bin/bash
# Round 2 (r2r): ABI 8 -- ipmc_pcn_run (the sampler's sampling loop in one C
# call): parity suite, the run-vs-per-sample tests, config 1 end to end, the
# sampler end to end at the headline size.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_run:300:python -u -m pytest tests/test_gpu_run.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "cfg1:300:python tools/probes/cfg1_e2e.py 1 > gpurun_out/cfg1_e2e.jsonl" \
  "e2e:300:python tools/sampler_e2e.py 65536 20 5 > gpurun_out/sampler_e2e.jsonl" \
  "stuart:300:python examples/stuart_examples.py 4096 > gpurun_out/example_stuart.jsonl"
