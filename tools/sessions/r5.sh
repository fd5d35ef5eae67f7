#!/bin/bash
# Round-5 GPU sessions: bash tools/sessions/r5.sh <name>
# Every GPU step has its own time limit.  A step that faults, aborts or times
# out ends the session (tests_ok lets pytest's "some tests failed" (rc 1)
# through, so one red assertion does not hide the rest of the session).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5
mkdir -p $O
export PYTHONUNBUFFERED=1
export IPMC_RECORD_DIR=$O
tests_ok() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
PYT="python -u -m pytest -v --timeout 600 --timeout-method thread"
case "$1" in
  s1)
    # paired FMA / REFERENCE accept streams on the benched problems, then the line
    tests_ok timeout -k 10 600 $PYT tests/test_gpu_paired_streams.py > $O/pytest_paired.log 2>&1
    timeout -k 10 600 python bench.py > $O/bench_s1.json 2> $O/bench_s1.err &&
    timeout -k 10 120 hipcc --offload-arch=gfx950 -O2 tools/probes/bpermute_exec_probe.hip -o $O/bp 2> /dev/null &&
    timeout -k 10 30 $O/bp > $O/bpermute_exec_probe.txt &&
    timeout -k 10 300 python tools/probes/spec_tree_debug.py bur128 > $O/walk_shfl_product.txt 2>&1 &&
    IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/walkshfl/libipmc.so timeout -k 10 300 \
        python tools/probes/spec_tree_debug.py bur128 > $O/walk_shfl_variant.txt 2>&1 &&
    for i in 1 2; do
      timeout -k 10 120 python tools/probes/arith_kernel_probe.py product >> $O/arith_waves_ab.jsonl &&
      IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/w2ref/libipmc.so timeout -k 10 120 \
          python tools/probes/arith_kernel_probe.py w2ref >> $O/arith_waves_ab.jsonl &&
      IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/w2fma/libipmc.so timeout -k 10 120 \
          python tools/probes/arith_kernel_probe.py w2fma >> $O/arith_waves_ab.jsonl || exit $?
    done
    ;;
  *)
    echo "unknown session $1"; exit 2
    ;;
esac
