#!/bin/bash
# Auto speculation on the DPP layout: GPU suite, then small ensembles up to 8 192 chains.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "suite:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider" \
  "small:500:python tools/probes/small_ensembles.py > gpurun_out/small_ensembles.jsonl"
