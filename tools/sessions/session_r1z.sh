#!/bin/bash
# rocprofv3 kernel statistics of the other configs (cross-check of config_bench's HIP-event times).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "stats_cfg:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg -o run -- python tools/config_bench.py cfg2 cfg4 cfg4full cfg5 ts6 ts36 > gpurun_out/configs_z.jsonl"
