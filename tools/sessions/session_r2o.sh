#!/bin/bash
# Round 2 (r2o): Lorenz-63 (config 2) speculative sweep: stall breakdown at
# speculation width 16 (1 wave per SIMD) and 32 (2 waves), after the fused
# k-sum; parity of the small kernels.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
tools/gpu_session.sh \
  "pytest_small:300:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k 'small or l63 or L63 or linear or speculative'" \
  "cfg2:300:python tools/config_bench.py cfg2@128 cfg2@128~8 cfg2@128~32 > gpurun_out/cfg2.jsonl" \
  "sq16:200:rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_cfg2_16 -o run -- python tools/config_bench.py cfg2@128" \
  "sq32:200:rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_cfg2_32 -o run -- python tools/config_bench.py cfg2@128~32"
