#!/bin/bash
# Round 2 re-entry: full GPU suite at HEAD (ABI 7), smoke, the bench line and
# its rocprofv3 kernel statistics.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "bench_prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --no-cpu > gpurun_out/bench_prof_line.json"
