#!/bin/bash
# Stall breakdown (SQ counters) of the Burgers (cfg 4, 2 048 chains) and two-scale (K=6 J=4) sweeps.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
tools/gpu_session.sh \
  "sq_bur:200:rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sq_bur -o run -- python tools/config_bench.py cfg4" \
  "sq_ts:200:rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sq_ts -o run -- python tools/config_bench.py ts6" \
  "sq_l96:200:rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sq_l96 -o run -- python bench.py --steps 5 --warmup 1 --no-cpu --no-extra"
