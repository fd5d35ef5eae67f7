#!/bin/bash
# bench.py N-rank rehearsal (2 ranks, gloo, one GPU) and the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_dist:400:python -u -m pytest tests/test_gpu_bench_dist.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf" \
  "bench:300:python bench.py > gpurun_out/bench_line.json"
