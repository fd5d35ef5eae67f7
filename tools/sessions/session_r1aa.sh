#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh "pytest_edges:300:python -u -m pytest tests/test_gpu_sampler_edges.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf"
