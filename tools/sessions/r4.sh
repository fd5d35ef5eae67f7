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
  *) echo "unknown session $1"; exit 2 ;;
esac
