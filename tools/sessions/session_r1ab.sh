#!/bin/bash
# Burgers layouts after the loop split and v_max: 8 cells x 32 lanes (default) vs 4 cells x 64 lanes.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh "lay:300:python tools/config_bench.py cfg4 cfg4:64 cfg4cfl cfg4cfl:64 cfg4full cfg4full:64 > gpurun_out/bur_layouts.jsonl"
