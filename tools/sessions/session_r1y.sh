#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh "ex_burgers:400:python examples/burgers_beta.py 1024 > gpurun_out/example_burgers_beta.json"
