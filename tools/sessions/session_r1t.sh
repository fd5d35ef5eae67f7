#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh "d2h:200:python tools/probes/d2h_probe.py > gpurun_out/d2h_probe.txt"
