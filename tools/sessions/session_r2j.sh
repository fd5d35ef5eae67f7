#!/bin/bash
# Round 2: spill-free sweep kernels (the proposal's Philox slots recomputed per
# step instead of hoisted and spilled around G; register floor 104), packed
# fp32 d=40 at 2 lanes per chain, packed-fp32 occupancy <= 256 registers.
# Parity suite, smoke, scans, configs, the bench line with its rocprofv3
# statistics and the PMC passes of both headline kernels.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra"
B32="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra --dtype f32"
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "scan40_65k:200:python tools/lanes_scan.py 65536 40 2000" \
  "scan40_8k:200:python tools/lanes_scan.py 8192 40 2000" \
  "configs:500:python tools/config_bench.py cfg2@128 cfg4 cfg4full cfg5 ts6 ts36 > gpurun_out/configs.jsonl" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "stats:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python bench.py --steps 20 --warmup 3 --no-cpu" \
  "fetch64:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/fetch -o run -- $B" \
  "write64:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/write -o run -- $B" \
  "sq64:200:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc64/sq -o run -- $B" \
  "fetch32:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/fetch -o run -- $B32" \
  "write32:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/write -o run -- $B32" \
  "sq32:200:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc32/sq -o run -- $B32" \
  "e2e:300:python tools/sampler_e2e.py 65536 20 5 > gpurun_out/sampler_e2e.jsonl"
