#!/bin/bash
# Round 2 (r2l): fp64 d=40 at 2 lanes per chain (spill-free since the per-step
# slot base): parity suite, smoke, the bench line, rocprofv3 statistics, PMC
# passes of the fp64 headline kernel, end to end.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra"
tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "scan40_65k:200:python tools/lanes_scan.py 65536 40 2000" \
  "bench:300:python bench.py > gpurun_out/bench_line.json" \
  "stats:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python bench.py --steps 20 --warmup 3 --no-cpu" \
  "fetch64:200:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/fetch -o run -- $B" \
  "write64:200:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/write -o run -- $B" \
  "sq64:200:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc64/sq -o run -- $B" \
  "e2e:300:python tools/sampler_e2e.py 65536 20 5 > gpurun_out/sampler_e2e.jsonl"
