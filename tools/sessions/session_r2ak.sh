#!/bin/bash
# Round 2 (r2ak): final tree (the product library rebuilt after the r2aj
# experiment was reverted): the whole GPU parity suite, smoke, the bench line,
# rocprofv3 statistics of the bench command, the drop-in API end to end and
# every config.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "stats:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python bench.py --steps 20 --warmup 3 --no-cpu" \
  "e2e:300:python tools/sampler_e2e.py 65536 20 5 > gpurun_out/sampler_e2e.jsonl" \
  "configs:500:python tools/config_bench.py cfg2@128 cfg4 cfg4visc cfg4cfl cfg4full cfg5 ts6 ts36 l96x1@256 l96x64@256 l96x1024@64 > gpurun_out/configs.jsonl"
