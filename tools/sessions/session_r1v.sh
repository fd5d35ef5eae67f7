#!/bin/bash
# SQ stall breakdown of the current Burgers sweep (cfg 4, 2 048 and 16 384 chains).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
tools/gpu_session.sh \
  "sq_bur:200:rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sq_bur2 -o run -- python tools/config_bench.py cfg4" \
  "sq_burfull:200:rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sq_burfull -o run -- python tools/config_bench.py cfg4full"
