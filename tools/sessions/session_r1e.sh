#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra"
tools/gpu_session.sh \
  "list:120:rocprofv3 -L > gpurun_out/counters.txt 2>&1" \
  "stats:600:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- $B" \
  "fetch:600:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- $B" \
  "write:600:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- $B" \
  "sq:600:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- $B"
