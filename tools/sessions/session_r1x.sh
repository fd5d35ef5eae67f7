#!/bin/bash
# Full GPU suite on the current tree, smoke, and the two reference-workflow examples.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "ex_lorenz:300:python examples/lorenz_thesis.py 1024 > gpurun_out/example_lorenz_thesis.json" \
  "ex_burgers:300:python examples/burgers_beta.py 1024 > gpurun_out/example_burgers_beta.json"
