#!/bin/bash
# Round-4 GPU sessions: bash tools/sessions/r4.sh <name>
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r4
mkdir -p $O
export PYTHONUNBUFFERED=1
case "$1" in
  explore)
    timeout -k 10 120 python tools/posterior_agreement.py chaos > $O/chaos.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.2 >> $O/explore.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.4 >> $O/explore.jsonl &&
    timeout -k 10 420 python tools/posterior_agreement.py prec 16384 20 50 0.2 >> $O/explore.jsonl
    ;;
  s1)
    # new GPU tests (host library == device draws, bench rehearsals), the new
    # bench line, then the posterior exploration
    timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
        tests/test_gpu_hostloop.py tests/test_gpu_bench_dist.py > $O/pytest_s1.log 2>&1 &&
    timeout -k 10 400 python bench.py > $O/bench_s1.json 2> $O/bench_s1.err &&
    timeout -k 10 120 python tools/posterior_agreement.py chaos > $O/chaos.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.2 >> $O/explore.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.4 >> $O/explore.jsonl &&
    timeout -k 10 420 python tools/posterior_agreement.py prec 16384 20 50 0.2 >> $O/explore.jsonl
    ;;
  *) echo "unknown session $1"; exit 2 ;;
esac
