#!/bin/bash
# Round-1 measurement refresh on the current build: parity suite, smoke, bench
# line, rocprofv3 kernel stats and PMC passes of the headline kernel (f64, f32),
# every config, end-to-end sampler throughput.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra"
B32="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra --dtype f32"
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "stats:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python bench.py --steps 20 --warmup 3 --no-cpu" \
  "fetch64:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/fetch -o run -- $B" \
  "write64:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/write -o run -- $B" \
  "sq64:200:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc64/sq -o run -- $B" \
  "fetch32:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/fetch -o run -- $B32" \
  "write32:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/write -o run -- $B32" \
  "sq32:200:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc32/sq -o run -- $B32" \
  "configs:500:python tools/config_bench.py cfg2 cfg2@128 cfg4 cfg4full cfg4cfl cfg4visc cfg5 ts6 ts36 l96x1 l96x64 l96x1024 > gpurun_out/configs.jsonl" \
  "e2e:300:python tools/sampler_e2e.py 65536 20 5 > gpurun_out/sampler_e2e.jsonl"
