#!/bin/bash
# Final-tree validation after the layout rule and block-wide speculation: GPU suite, smoke, bench line, rocprofv3 statistics.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "suite:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -p no:cacheprovider" \
  "smoke:180:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench:400:python bench.py > gpurun_out/bench_line.json" \
  "stats:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python bench.py --steps 20 --warmup 3 --no-cpu"
