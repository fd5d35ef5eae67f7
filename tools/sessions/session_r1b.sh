#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "lanes_scan:600:python tools/lanes_scan.py 65536" \
  "bench:900:python bench.py --steps 20 --warmup 3" \
  "rocprof:900:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o bench -- python bench.py --steps 20 --warmup 3 --no-cpu"
