#!/bin/bash
# Round-5 GPU sessions: bash tools/sessions/r5.sh <name>
# Every GPU step has its own time limit.  A step that faults, aborts or times
# out ends the session (tests_ok lets pytest's "some tests failed" (rc 1)
# through, so one red assertion does not hide the rest of the session).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5
mkdir -p $O
export PYTHONUNBUFFERED=1
export IPMC_RECORD_DIR=$O
tests_ok() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
PYT="python -u -m pytest -v --timeout 600 --timeout-method thread"
case "$1" in
  s1)
    # paired FMA / REFERENCE accept streams on the benched problems, then the line
    tests_ok timeout -k 10 600 $PYT tests/test_gpu_paired_streams.py > $O/pytest_paired.log 2>&1
    timeout -k 10 600 python bench.py > $O/bench_s1.json 2> $O/bench_s1.err &&
    timeout -k 10 120 hipcc --offload-arch=gfx950 -O2 tools/probes/bpermute_exec_probe.hip -o $O/bp 2> /dev/null &&
    timeout -k 10 30 $O/bp > $O/bpermute_exec_probe.txt &&
    timeout -k 10 300 python tools/probes/spec_tree_debug.py bur128 > $O/walk_shfl_product.txt 2>&1 &&
    IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/walkshfl/libipmc.so timeout -k 10 300 \
        python tools/probes/spec_tree_debug.py bur128 > $O/walk_shfl_variant.txt 2>&1 &&
    for i in 1 2; do
      timeout -k 10 120 python tools/probes/arith_kernel_probe.py product >> $O/arith_waves_ab.jsonl &&
      IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/w2ref/libipmc.so timeout -k 10 120 \
          python tools/probes/arith_kernel_probe.py w2ref >> $O/arith_waves_ab.jsonl &&
      IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/w2fma/libipmc.so timeout -k 10 120 \
          python tools/probes/arith_kernel_probe.py w2fma >> $O/arith_waves_ab.jsonl || exit $?
    done
    ;;
  s2)
    # the whole GPU suite on the tree (REFERENCE arith at two waves, the K/3
    # two-scale ring, the paired-stream tests), the walk probe with the read
    # under the first lane's branch, the two-scale K=36 layout / halo A/B
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_s2.log 2>&1
    IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/walkshfl2/libipmc.so timeout -k 10 300 \
        python tools/probes/spec_tree_debug.py bur128 > $O/walk_shfl_first_lane.txt 2>&1 &&
    for i in 1 2; do
      timeout -k 10 300 python tools/config_bench.py ts36 ts36:12 >> $O/ts36_layouts.jsonl &&
      IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/tslds/libipmc.so timeout -k 10 300 \
          python tools/config_bench.py ts36 ts36:12 | sed 's/^{/{"variant": "lds_halo", /' >> $O/ts36_layouts.jsonl || exit $?
    done
    ;;
  s3)
    # in-wave speculative rounds resolved in parallel (L96, Burgers, two-scale):
    # the whole suite, then the speculation rows and the reference studies
    # against the walk build (variants/prevwalk = the previous commit)
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_s3.log 2>&1
    R="l96mx1@256 l96mx64@256 l96mx1024@256 l96x1@256 l96x64@256 cfg2@16384"
    for i in 1 2; do
      for lib in "" ip_mcmc_amd/lib/variants/prevwalk/libipmc.so; do
        IPMC_LIB_PATH=$lib timeout -k 10 300 python tools/config_bench.py $R | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin]" \
          >> $O/walk_ab_rows.jsonl &&
        IPMC_LIB_PATH=$lib timeout -k 10 200 python tools/probes/burgers_spec_probe.py 1024 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin if l.startswith('{')]" \
          >> $O/walk_ab_burgers.jsonl &&
        IPMC_LIB_PATH=$lib timeout -k 10 200 python tools/probes/burgers_spec_probe.py 1 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin if l.startswith('{')]" \
          >> $O/walk_ab_burgers.jsonl &&
        IPMC_LIB_PATH=$lib timeout -k 10 300 python examples/lorenz_thesis.py 1024 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin if l.startswith('{')]" \
          >> $O/walk_ab_lorenz.jsonl || exit 1
      done
    done
    ;;
  s4)
    # the fp64 Lorenz-96 sweep with its lane state parked in LDS across G at
    # two waves per SIMD (variants/park) against the product (one wave for
    # FMA), FMA and REFERENCE arith, interleaved three times; PMC traffic of both
    V=ip_mcmc_amd/lib/variants/park/libipmc.so
    B="python bench.py --kernel-only --no-cpu --steps 5 --warmup 1"
    SQC="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    for i in 1 2 3; do
      timeout -k 10 120 python tools/probes/arith_kernel_probe.py product >> $O/park_ab.jsonl &&
      IPMC_LIB_PATH=$V timeout -k 10 120 python tools/probes/arith_kernel_probe.py park >> $O/park_ab.jsonl || exit 1
    done &&
    for lib in product park; do
      L=""; [ $lib = park ] && L=$V
      IPMC_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
          -d $O/pmc_$lib/fetch -o run -- $B > /dev/null &&
      IPMC_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
          -d $O/pmc_$lib/write -o run -- $B > /dev/null &&
      IPMC_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv \
          -d $O/pmc_$lib/sq -o run -- $B > /dev/null &&
      python tools/pmc_summarize.py $O/pmc_$lib f64 65536 $O/pmc_l96_f64_$lib.json 6 || exit 1
    done
    ;;
  s5)
    # the tree with the parked fp64 sweep at two waves, the device ordered sum
    # (ABI 12): the whole suite, smoke, the default line
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_s5.log 2>&1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_s5.txt 2>&1 &&
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_s5_k20.json 2> $O/bench_s5_k20.err &&
    timeout -k 10 600 python bench.py --no-configs --no-cpu > $O/bench_s5_k200.json 2> $O/bench_s5_k200.err
    ;;
  s6)
    # the LDS-staged device ordered sum: its test, the probe, the driver's line
    tests_ok timeout -k 10 600 $PYT tests/test_gpu_shard.py > $O/pytest_s6.log 2>&1
    timeout -k 10 120 python tools/probes/ordered_sum_probe.py > $O/ordered_sum_probe.jsonl &&
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_s6_k20.json 2> $O/bench_s6_k20.err
    ;;
  final)
    # the final tree: the whole suite and smoke, then the published line with
    # its same-box profiles -- three PMC passes of the kernel leg (bench
    # --kernel-only), the line reading them (default K/W and the driver's
    # K=20 W=5), a kernel trace + stats of the kernel leg restricted to the
    # timed launches, the f32 PMC passes
    B="python bench.py --kernel-only --no-cpu --steps 5 --warmup 1"
    SQC="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_final.log 2>&1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final.txt 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc64/fetch -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc64/write -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $O/pmc64/sq -o run -- $B > /dev/null &&
    python tools/pmc_summarize.py $O/pmc64 f64 65536 $O/pmc_l96_f64.json 6 &&
    timeout -k 10 600 python bench.py --pmc-file $O/pmc_l96_f64.json > $O/bench_line.json 2> $O/bench_line.err &&
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 --pmc-file $O/pmc_l96_f64.json > $O/bench_line_k20.json \
        2> $O/bench_line_k20.err &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
        python bench.py --kernel-only --no-cpu > $O/bench_kernel_only.json 2> $O/bench_kernel_only.err &&
    python tools/trace_summary.py $O/trace 200 10 $O/bench_line.json > $O/bench_kernel_trace_summary.json &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc32/fetch -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc32/write -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $O/pmc32/sq -o run -- $B --dtype f32 > /dev/null &&
    python tools/pmc_summarize.py $O/pmc32 f32 65536 $O/pmc_l96_f32.json 6
    ;;
  e2etrace)
    # kernel + copy trace of the driver's K=20 line (end-to-end leg included):
    # per-launch sweep times inside run() against the kernel leg's, the gaps
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/e2etrace -o run -- \
      python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-configs --no-parity > $O/e2etrace.json \
      2> $O/e2etrace.err
    ;;
  settle)
    # end-to-end legs with the clocks settled before their timed region, weak
    # scaling by default: the N-rank and shard tests, the driver's K=20 line,
    # then the kernel + copy trace of a short line
    tests_ok timeout -k 10 900 $PYT tests/test_gpu_bench_dist.py tests/test_gpu_shard.py > $O/pytest_settle.log 2>&1
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 --pmc-file profiles/r5/pmc_l96_f64.json \
      > $O/bench_settle_k20.json 2> $O/bench_settle_k20.err &&
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/e2etrace_settle -o run -- \
      python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-configs --no-parity > $O/e2etrace_settle.json \
      2> $O/e2etrace_settle.err
    ;;
  f32ab)
    # the packed fp32 headline sweep: the round-5-start build of its unit
    # (variants/r5start, identical ISA by hipcc -S) against the product,
    # interleaved three times -- is the 1.70 -> 1.95 ms move the box or the code?
    for i in 1 2 3; do
      timeout -k 10 120 python tools/probes/arith_kernel_probe.py product 40 f32 >> $O/f32_ab.jsonl &&
      IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/r5start/libipmc.so timeout -k 10 120 \
          python tools/probes/arith_kernel_probe.py r5start 40 f32 >> $O/f32_ab.jsonl || exit 1
    done
    ;;
  s7)
    # block-sum posterior mean (ABI 13), weak-scaling default, settled e2e legs:
    # the whole suite, smoke, the fp32 A/B, the driver's K=20 line, a trace
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_s7.log 2>&1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_s7.txt 2>&1 &&
    bash tools/sessions/r5.sh f32ab &&
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 --pmc-file profiles/r5/pmc_l96_f64.json \
      > $O/bench_s7_k20.json 2> $O/bench_s7_k20.err &&
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/e2etrace_s7 -o run -- \
      python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-configs --no-parity > $O/e2etrace_s7.json \
      2> $O/e2etrace_s7.err
    ;;
  s9)
    # results='device' (value with the data in HBM), block sums over ranks on
    # the device: the sampler / shard / N-rank tests, the driver's K=20 line
    tests_ok timeout -k 10 900 $PYT tests/test_gpu_shard.py tests/test_gpu_bench_dist.py tests/test_gpu_run.py \
      tests/test_gpu_sampler_edges.py tests/test_gpu_hostloop.py > $O/pytest_s9.log 2>&1
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 --pmc-file profiles/r5/pmc_l96_f64.json \
      > $O/bench_s9_k20.json 2> $O/bench_s9_k20.err
    ;;
  rows)
    # the configs' and the small ensembles' rows and the reference studies on the final tree
    timeout -k 10 600 python tools/config_bench.py cfg2@16384 cfg4 cfg4full cfg5 ts6 ts36 > $O/configs_final.jsonl &&
    timeout -k 10 300 python tools/config_bench.py l96mx1@256 l96mx64@256 l96mx1024@256 l96x1@256 l96x64@256 \
        > $O/spec_final.jsonl &&
    for args in "burgers_beta.py 1024" "burgers_beta.py 1" "lorenz_thesis.py 1024" "lorenz_thesis.py 1" \
                "lorenz63_config2.py" "stuart_reference.py"; do
      set -- $args
      timeout -k 10 300 python examples/$1 ${2:-} > $O/ex_tmp.jsonl || exit 1
      python -c "import json,sys;[print(json.dumps(dict(json.loads(l),example='$1',arg='${2:-}'))) for l in open('$O/ex_tmp.jsonl') if l.startswith('{')]" >> $O/examples_final.jsonl || exit 1
    done
    ;;
  *)
    echo "unknown session $1"; exit 2
    ;;
esac
