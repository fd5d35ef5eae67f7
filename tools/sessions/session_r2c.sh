#!/bin/bash
# Round 2: parity after non-diagonal priors (prior_chol in every sweep kernel)
# and the Burgers chain fixture; the bench line (headline kernel unchanged).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_new:300:python -u -m pytest tests/test_gpu_parity.py tests/test_chainio.py tests/test_gpu_diag.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'dense or burgers_chain or back_to_back or recomputes or longer_than'" \
  "pytest_gpu:700:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "bench:300:python bench.py --no-cpu > gpurun_out/bench_line.json"
