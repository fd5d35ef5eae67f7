#!/bin/bash
# fp32 vs fp64 tolerance sweep (config 5, Lorenz-96 d=256) and a bench-argument sanity run.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "precision:500:python tools/precision_sweep.py 16384 200 > gpurun_out/precision_sweep.jsonl"
