#!/bin/bash
# Round 2 (r2al): PMC passes of both headline kernels on the final tree (one
# counter group per run), summarised by tools/pmc_summarize.py into
# profiles/r2/pmc_l96_{f64,f32}.json for the bench line's roofline.traffic.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra"
B32="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra --dtype f32"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
tools/gpu_session.sh \
  "fetch64:120:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/fetch -o run -- $B" \
  "write64:120:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/write -o run -- $B" \
  "sq64:120:rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/pmc64/sq -o run -- $B" \
  "fetch32:120:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/fetch -o run -- $B32" \
  "write32:120:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/write -o run -- $B32" \
  "sq32:120:rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/pmc32/sq -o run -- $B32"
