#!/bin/bash
# Round-6 GPU sessions: bash tools/sessions/r6.sh <name>
# Every GPU step has its own time limit.  A step that faults, aborts or times
# out ends the session (tests_ok lets pytest's "some tests failed" (rc 1)
# through, so one red assertion does not hide the rest of the session).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1
export IPMC_RECORD_DIR=$O
tests_ok() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
PYT="python -u -m pytest -v --timeout 600 --timeout-method thread"
SQC="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
# the metric's 8-GPU share on one GPU: 8 192 chains (global ids 7*8192..), the driver's K = 20
SHARD="python bench.py --chains 8192 --scaling strong --steps 20 --warmup 5 --no-cpu --no-extra --no-configs --no-parity"
case "$1" in
  shard0)
    # the 8 192-chain strong shard on the round-6 starting tree: the line twice,
    # a kernel trace of the end-to-end leg, an SQ pass of the kernel leg
    for i in 1 2; do
      timeout -k 10 300 $SHARD >> $O/shard0_lines.jsonl 2>> $O/shard0.err || exit $?
    done &&
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/shard0_trace -o run -- \
      $SHARD > $O/shard0_trace.json 2> $O/shard0_trace.err &&
    python tools/e2e_trace_summary.py $O/shard0_trace > $O/shard0_trace_summary.json &&
    timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $O/shard0_sq -o run -- \
      $SHARD --kernel-only > /dev/null 2>> $O/shard0.err &&
    python tools/sq_summarize.py $O/shard0_sq 'sweep_kernel' > $O/shard0_sq.json
    ;;
  ab8)
    # the 8 192-chain shard's kernel (d=40 on 8 lanes, one 20-step launch):
    # product vs halo-first component order (hf), one-wave target (w1), RK
    # loop unrolled by 2 (u2), interleaved twice; the headline kernel for hf
    for i in 1 2; do
      for v in product hf w1 u2; do
        L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
        IPMC_LIB_PATH=$L timeout -k 10 120 python tools/probes/shard_kernel_probe.py $v >> $O/ab8.jsonl || exit 1
      done
    done &&
    for v in product hf; do
      L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
      IPMC_LIB_PATH=$L timeout -k 10 120 python tools/probes/arith_kernel_probe.py $v >> $O/ab8_headline.jsonl || exit 1
    done
    ;;
  s1)
    # strong scaling by default, rank-local u_0, fp32/fp64 at r = 0.5: the
    # N-rank and shard tests, the new tolerance test; the host profile of the
    # 8 192-chain end-to-end leg
    tests_ok timeout -k 10 900 $PYT tests/test_gpu_bench_dist.py tests/test_gpu_shard.py \
      "tests/test_gpu_arith_agreement.py::test_fp32_and_fp64_posteriors_agree_at_the_references_noise_level" \
      > $O/pytest_s1.log 2>&1
    timeout -k 10 200 python tools/probes/shard_e2e_profile.py 8192 20 3 s1 >> $O/shard_e2e.jsonl 2> $O/shard_e2e_prof_s1.txt
    ;;
  ab9)
    # x(0)'s loads waited for before the RK loop (pw: 129 -> 127 instructions
    # per RK4 step at 8 lanes) and two RK4 steps per iteration (pwp: 126.5),
    # against the product, interleaved three times; the headline kernel; the
    # 8 192-chain end-to-end leg with the cached constants, product vs pwp
    for i in 1 2 3; do
      for v in product pw pwp; do
        L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
        IPMC_LIB_PATH=$L timeout -k 10 120 python tools/probes/shard_kernel_probe.py $v >> $O/ab9.jsonl || exit 1
      done
    done &&
    for v in product pw; do
      L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
      IPMC_LIB_PATH=$L timeout -k 10 120 python tools/probes/arith_kernel_probe.py $v >> $O/ab9_headline.jsonl || exit 1
    done &&
    for i in 1 2; do
      for v in product pwp; do
        L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
        IPMC_LIB_PATH=$L timeout -k 10 200 python tools/probes/shard_e2e_profile.py 8192 20 3 $v >> $O/ab9_e2e.jsonl \
          2> /dev/null || exit 1
      done
    done
    ;;
  ab10)
    # R RK4 steps per loop iteration: R = 2 up to M = 10 (r2m10), R = 4 up to
    # M = 10 (r4m10), R = 2 up to M = 20 (r2m20, the headline kernel too), at
    # the per-GPU shares of N = 8 / 4 / 2 (8 192 / 16 384 / 32 768 chains, one
    # wave per SIMD each) and the headline, interleaved twice
    for i in 1 2; do
      for c in 8192 16384 32768; do
        for v in product r2m10 r4m10 r2m20; do
          L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
          IPMC_LIB_PATH=$L timeout -k 10 120 python tools/probes/shard_kernel_probe.py $v 20 $c 2 >> $O/ab10.jsonl || exit 1
        done
      done
      for v in product r2m20; do
        L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
        IPMC_LIB_PATH=$L timeout -k 10 120 python tools/probes/arith_kernel_probe.py $v >> $O/ab10_headline.jsonl || exit 1
      done
    done
    ;;
  ab11)
    # what keep="moments"' per-step sums cost the 8 192 / 65 536-chain sweeps (sums vs none, interleaved)
    for i in 1 2 3; do
      for c in 8192 65536; do
        timeout -k 10 120 python tools/probes/shard_kernel_probe.py nosums 20 $c 2 >> $O/ab11.jsonl &&
        timeout -k 10 120 python tools/probes/shard_kernel_probe.py sums 20 $c 2 sums >> $O/ab11.jsonl || exit 1
      done
    done
    ;;
  s3)
    bash tools/sessions/r6.sh ab10 && bash tools/sessions/r6.sh ab11
    ;;
  s4)
    # the tree with R = 4 RK4 steps per iteration up to M = 10: the whole suite,
    # smoke, the per-GPU shares at K = 20
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_s4.log 2>&1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_s4.txt 2>&1 &&
    bash tools/sessions/r6.sh shards
    ;;
  prof)
    # host-side profile (microseconds per function) of the 8 192-chain end-to-end leg
    timeout -k 10 200 python tools/probes/shard_e2e_profile.py 8192 20 4 prof >> $O/shard_e2e_prof.jsonl \
      2> $O/shard_e2e_prof_us.txt
    ;;
  s5)
    # the host trims: the 8 192-chain profile again, then the final session
    bash tools/sessions/r6.sh prof && bash tools/sessions/r6.sh shards && bash tools/sessions/r6.sh final
    ;;
  s6)
    # l96_stage back to its round-5 form (the packed fp32 headline's ISA equals
    # round 5's again): the f32 / f64 headline kernel legs, the 8 192-chain
    # shard kernel, a kernel trace of the driver's K = 20 line (end-to-end
    # sweep vs kernel leg), the new one-rank RCCL bench test
    for i in 1 2; do
      timeout -k 10 120 python tools/probes/arith_kernel_probe.py s6 40 f32 >> $O/s6_f32.jsonl &&
      timeout -k 10 120 python tools/probes/arith_kernel_probe.py s6 40 f64 >> $O/s6_f64.jsonl &&
      timeout -k 10 120 python tools/probes/shard_kernel_probe.py s6 20 8192 2 >> $O/s6_shard.jsonl || exit 1
    done &&
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/e2etrace_s6 -o run -- \
      python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-configs --no-parity > $O/e2etrace_s6.json \
      2> $O/e2etrace_s6.err &&
    python tools/e2e_trace_summary.py $O/e2etrace_s6 > $O/e2etrace_s6_summary.json &&
    { tests_ok timeout -k 10 600 $PYT tests/test_gpu_bench_dist.py -k one_rank > $O/pytest_s6.log 2>&1; }
    ;;
  s7)
    # block sums queued before run()'s one synchronisation (pre_sync): the
    # sharding / sampler tests, the 8 192-chain end-to-end profile, the shares
    tests_ok timeout -k 10 900 $PYT tests/test_gpu_shard.py tests/test_gpu_run.py tests/test_gpu_sampler_edges.py \
      tests/test_gpu_bench_dist.py > $O/pytest_s7.log 2>&1
    timeout -k 10 200 python tools/probes/shard_e2e_profile.py 8192 20 4 s7 >> $O/shard_e2e_s7.jsonl \
      2> $O/shard_e2e_prof_s7.txt &&
    SHARDS_TAG=_s7 bash tools/sessions/r6.sh shards
    ;;
  s8)
    # RK4 step counts that are not a multiple of the 4-step unroll
    tests_ok timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "multiple_of_the_unroll or interleaved_8 or forward_and_potential" \
      > $O/pytest_s8.log 2>&1
    ;;
  ab12)
    # the packed fp32 headline kernel: product vs the mid-round source (the RK4
    # step as a lambda in a counted loop, 6a006ca: other VGPR numbering) vs the
    # l96_stage rewrite alone (stagecopy: the product's RK loop byte for byte),
    # interleaved three times
    for i in 1 2 3; do
      for v in product r6mid stagecopy; do
        L=""; [ $v != product ] && L=ip_mcmc_amd/lib/variants/$v/libipmc.so
        IPMC_LIB_PATH=$L timeout -k 10 120 python tools/probes/arith_kernel_probe.py $v 40 f32 >> $O/ab12_f32.jsonl || exit 1
      done
    done
    ;;
  s9)
    # the examples (config 5 with a rank-local u_0) and the sharding tests on the final tree
    tests_ok timeout -k 10 900 $PYT tests/test_gpu_examples.py tests/test_gpu_shard.py > $O/pytest_s9.log 2>&1
    ;;
  suite)
    # the whole GPU suite and smoke on the tree as it stands
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_suite.log 2>&1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_suite.txt 2>&1
    ;;
  gloo8)
    # the driver's 8-GPU line rehearsed with gloo, all eight ranks on the one
    # GPU (strong scaling by default: 65 536 chains over the node under
    # BASELINE's metric, 8 192 per rank; the weak figure in extra)
    timeout -k 10 900 python bench.py --gpus 8 --steps 20 --warmup 5 --dist-backend gloo --share-device --no-cpu \
      --no-configs > $O/bench_gloo8.json 2> $O/bench_gloo8.err
    ;;
  s2)
    # ab9, then the shard tests with the one-rank RCCL group, the gloo 8-rank line
    bash tools/sessions/r6.sh ab9 &&
    { tests_ok timeout -k 10 600 $PYT tests/test_gpu_shard.py > $O/pytest_s2.log 2>&1; } &&
    bash tools/sessions/r6.sh gloo8
    ;;
  final)
    # the final tree: the whole suite and smoke, then the published line with
    # its same-box profiles -- three PMC passes of the kernel leg (bench
    # --kernel-only), the line reading them (default K/W and the driver's
    # K=20 W=5), a kernel trace + stats of the kernel leg restricted to the
    # timed launches, the f32 PMC passes
    B="python bench.py --kernel-only --no-cpu --steps 5 --warmup 1"
    SQ5="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    tests_ok timeout -k 10 1200 $PYT tests -m gpu > $O/pytest_gpu_final.log 2>&1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final.txt 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc64/fetch -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc64/write -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQ5 --kernel-trace --output-format csv -d $O/pmc64/sq -o run -- $B > /dev/null &&
    python tools/pmc_summarize.py $O/pmc64 f64 65536 $O/pmc_l96_f64.json 6 &&
    timeout -k 10 600 python bench.py --pmc-file $O/pmc_l96_f64.json > $O/bench_line.json 2> $O/bench_line.err &&
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 --pmc-file $O/pmc_l96_f64.json > $O/bench_line_k20.json \
        2> $O/bench_line_k20.err &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
        python bench.py --kernel-only --no-cpu > $O/bench_kernel_only.json 2> $O/bench_kernel_only.err &&
    python tools/trace_summary.py $O/trace 200 10 $O/bench_line.json > $O/bench_kernel_trace_summary.json &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc32/fetch -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc32/write -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQ5 --kernel-trace --output-format csv -d $O/pmc32/sq -o run -- $B --dtype f32 > /dev/null &&
    python tools/pmc_summarize.py $O/pmc32 f32 65536 $O/pmc_l96_f32.json 6
    ;;
  shards)
    # the per-GPU shares of the metric's 65 536 chains at N = 2, 4, 8 (strong
    # scaling), each on this one GPU at the driver's K = 20, twice
    for i in 1 2; do
      for c in 32768 16384 8192; do
        timeout -k 10 300 python bench.py --chains $c --steps 20 --warmup 5 --no-cpu --no-extra --no-configs \
          --no-parity >> $O/shards_k20${SHARDS_TAG:-}.jsonl 2>> $O/shards.err || exit 1
      done
    done
    ;;
  *)
    echo "unknown session $1"; exit 2
    ;;
esac
