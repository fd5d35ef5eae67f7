#!/bin/bash
# Sampler samples through page-locked host memory: API tests and end-to-end throughput.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_api:600:python -u -m pytest tests/test_gpu_parity.py tests/test_chainio.py tests/test_gpu_shard.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf -k 'sampler or chain or resume or shard or stream'" \
  "e2e:300:python tools/sampler_e2e.py 65536 20 5 > gpurun_out/sampler_e2e.jsonl"
