#!/bin/bash
# Round-4 GPU sessions: bash tools/sessions/r4.sh <name>
# Every GPU step has its own time limit and the steps are chained with &&.
# The A/B sessions load variant builds of libipmc.so (not kept in the tree;
# rebuild them on the CPU first):
#   l63scalar  tools/build_variant.sh l63scalar ipmc_api.hip -DIPMC_L63_PK=0
#   speck8     tools/build_variant.sh speck8 ipmc_api.hip -DIPMC_SPEC_K3=0
#   pathspec   make -C ip_mcmc_amd/csrc -j8 OBJDIR=../../build/variants/pathspec \
#                OUT=../lib/variants/pathspec/libipmc.so \
#                HOST_OUT=../../build/variants/pathspec/libipmc_host.so EXTRA=-DIPMC_SPEC_TREE=0
#   m095       the same with m095 and EXTRA=-DIPMC_SPEC_MEMORY=0.95f
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r4
mkdir -p $O
export PYTHONUNBUFFERED=1
case "$1" in
  explore)
    timeout -k 10 120 python tools/posterior_agreement.py chaos > $O/chaos.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.2 >> $O/explore.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.4 >> $O/explore.jsonl &&
    timeout -k 10 420 python tools/posterior_agreement.py prec 16384 20 50 0.2 >> $O/explore.jsonl
    ;;
  s1)
    # new GPU tests (host library == device draws, bench rehearsals), the new
    # bench line, then the posterior exploration
    timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
        tests/test_gpu_hostloop.py tests/test_gpu_bench_dist.py > $O/pytest_s1.log 2>&1 &&
    timeout -k 10 400 python bench.py > $O/bench_s1.json 2> $O/bench_s1.err &&
    timeout -k 10 120 python tools/posterior_agreement.py chaos > $O/chaos.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.2 >> $O/explore.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 40 50 0.4 >> $O/explore.jsonl &&
    timeout -k 10 420 python tools/posterior_agreement.py prec 16384 20 50 0.2 >> $O/explore.jsonl
    ;;
  s2)
    # the whole GPU suite, then the published line and its profiles from one
    # box: three PMC passes of the kernel leg (bench --kernel-only), the bench
    # line reading them, a rocprofv3 kernel trace + stats of the kernel leg
    # (same K/W as the line) and its summary, the f32 PMC passes
    B="python bench.py --kernel-only --no-cpu --steps 5 --warmup 1"
    SQC="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc64/fetch -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc64/write -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $O/pmc64/sq -o run -- $B > /dev/null &&
    python tools/pmc_summarize.py $O/pmc64 f64 65536 $O/pmc_l96_f64.json 6 &&
    timeout -k 10 600 python bench.py --pmc-file $O/pmc_l96_f64.json > $O/bench_line.json 2> $O/bench_line.err &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
        python bench.py --kernel-only --no-cpu > $O/bench_kernel_only.json 2> $O/bench_kernel_only.err &&
    python tools/trace_summary.py $O/trace 200 10 $O/bench_line.json > $O/bench_kernel_trace_summary.json &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc32/fetch -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc32/write -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $O/pmc32/sq -o run -- $B --dtype f32 > /dev/null &&
    python tools/pmc_summarize.py $O/pmc32 f32 65536 $O/pmc_l96_f32.json 6
    ;;
  s12)
    # everything the first box can give: the misfit-noise probe and a first
    # stationary arith comparison, the whole GPU suite (no -x: one statistical
    # failure must not hide the rest), the line with its same-box profiles,
    # then the config-5-shape precision comparison
    timeout -k 10 120 python tools/posterior_agreement.py chaos > $O/chaos.jsonl &&
    timeout -k 10 300 python tools/posterior_agreement.py arith 8192 48 50 0.2 >> $O/explore.jsonl &&
    { timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; } &&
    bash tools/sessions/r4.sh s2prof &&
    timeout -k 10 420 python tools/posterior_agreement.py prec 16384 24 50 0.2 >> $O/explore.jsonl
    ;;
  s2prof)
    B="python bench.py --kernel-only --no-cpu --steps 5 --warmup 1"
    SQC="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc64/fetch -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc64/write -o run -- $B > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $O/pmc64/sq -o run -- $B > /dev/null &&
    python tools/pmc_summarize.py $O/pmc64 f64 65536 $O/pmc_l96_f64.json 6 &&
    timeout -k 10 600 python bench.py --pmc-file $O/pmc_l96_f64.json > $O/bench_line.json 2> $O/bench_line.err &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
        python bench.py --kernel-only --no-cpu > $O/bench_kernel_only.json 2> $O/bench_kernel_only.err &&
    python tools/trace_summary.py $O/trace 200 10 $O/bench_line.json > $O/bench_kernel_trace_summary.json &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc32/fetch -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc32/write -o run -- $B --dtype f32 > /dev/null &&
    timeout -s KILL 120 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $O/pmc32/sq -o run -- $B --dtype f32 > /dev/null &&
    python tools/pmc_summarize.py $O/pmc32 f32 65536 $O/pmc_l96_f32.json 6
    ;;
  s3)
    # stationary-posterior calibration (noise level r, beta, run length) and
    # the Lorenz-63 fp32 packing A/B on config 2 (interleaved with the product)
    P="python tools/posterior_agreement.py"
    V=ip_mcmc_amd/lib/variants/l63scalar/libipmc.so
    for cfg in "1.0 0.2" "2.0 0.2" "1.0 0.5" "2.0 0.5"; do
      set -- $cfg
      timeout -k 10 200 $P arith 8192 48 50 $2 $1 nopair >> $O/calib_arith.jsonl || exit 1
    done &&
    timeout -k 10 300 $P arith 8192 96 50 0.3 1.0 nopair >> $O/calib_arith.jsonl &&
    timeout -k 10 300 $P prec 4096 24 50 0.3 2.0 nopair >> $O/calib_prec.jsonl &&
    timeout -k 10 300 $P prec 4096 24 50 0.3 4.0 nopair >> $O/calib_prec.jsonl &&
    timeout -k 10 200 python tools/config_bench.py cfg2 >> $O/l63_pk_ab.jsonl &&
    IPMC_LIB_PATH=$V timeout -k 10 200 python tools/config_bench.py cfg2 >> $O/l63_pk_ab.jsonl &&
    timeout -k 10 200 python tools/config_bench.py cfg2 >> $O/l63_pk_ab.jsonl &&
    IPMC_LIB_PATH=$V timeout -k 10 200 python tools/config_bench.py cfg2 >> $O/l63_pk_ab.jsonl &&
    timeout -k 10 200 python tools/config_bench.py ts36 ts36:36 ts36 ts36:36 >> $O/ts36_layouts.jsonl &&
    timeout -k 10 200 python tools/config_bench.py l96mx1@256 l96mx64@256 l96mx1024@256 l96x1@256 l96x64@256 >> $O/spec_mixing.jsonl &&
    timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread \
        tests/test_gpu_arith_agreement.py tests/test_gpu_tolerance.py > $O/pytest_stationary.log 2>&1
    ;;
  s4)
    # config 2 with the k = 3 specialised speculative sweep: A/B against the
    # generic-k variant (long launches, interleaved), one SQ pass per dtype;
    # then the whole GPU suite (the stationary tests record their numbers)
    # and the published line with its same-box profiles
    V=ip_mcmc_amd/lib/variants/speck8/libipmc.so
    SQS="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
    for i in 1 2; do
      timeout -k 10 200 python tools/config_bench.py cfg2@16384 >> $O/l63_k3_ab.jsonl &&
      IPMC_LIB_PATH=$V timeout -k 10 200 python tools/config_bench.py cfg2@16384 >> $O/l63_k3_ab.jsonl || exit 1
    done &&
    timeout -k 10 200 python tools/config_bench.py cfg2@16384:32 >> $O/l63_k3_ab.jsonl &&
    timeout -s KILL 90 rocprofv3 --pmc $SQS --kernel-trace --output-format csv -d $O/sq_cfg2/f64 -o run -- \
        python tools/config_bench.py cfg2@16384!f64 > /dev/null &&
    timeout -s KILL 90 rocprofv3 --pmc $SQS --kernel-trace --output-format csv -d $O/sq_cfg2/f32 -o run -- \
        python tools/config_bench.py cfg2@16384!f32 > /dev/null &&
    python tools/sq_summarize.py $O/sq_cfg2/f64 small_spec_kernel > $O/sq_cfg2_f64.json &&
    python tools/sq_summarize.py $O/sq_cfg2/f32 small_spec_kernel > $O/sq_cfg2_f32.json &&
    { IPMC_RECORD_DIR=$O timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_s4.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; } &&
    bash tools/sessions/r4.sh s2prof
    ;;
  s5)
    # Lorenz-63 fp32 packing A/B at the sampler's launch length (s3's was at
    # one step per launch: launch-bound), and the mixing-posterior small
    # ensembles without speculation (spec width 1) beside s3's speculative rows
    V=ip_mcmc_amd/lib/variants/l63scalar/libipmc.so
    for i in 1 2; do
      timeout -k 10 200 python tools/config_bench.py 'cfg2@16384!f32' >> $O/l63_pk_ab_long.jsonl &&
      IPMC_LIB_PATH=$V timeout -k 10 200 python tools/config_bench.py 'cfg2@16384!f32' >> $O/l63_pk_ab_long.jsonl || exit 1
    done &&
    timeout -k 10 300 python tools/config_bench.py l96mx1~1@256 l96mx64~1@256 l96mx1024~1@256 >> $O/spec_mixing_nospec.jsonl
    ;;
  s6)
    # speculation trees: the speculative parity tests first (stop on a
    # failure), then the whole suite, then the small-ensemble rows on the
    # mixing posterior and the accept-nothing problem, config 2 and the
    # sequential Burgers / two-scale sweeps against the two-path build
    V=ip_mcmc_amd/lib/variants/pathspec/libipmc.so
    timeout -k 10 300 python tools/probes/spec_tree_debug.py > $O/spec_tree_debug.txt 2>&1 &&
    timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
        -k "speculative or dense_prior or small_models" > $O/pytest_tree_spec.log 2>&1 &&
    { timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_s6.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; } &&
    R="l96mx1@256 l96mx64@256 l96mx1024@256 l96x1@256 l96x64@256" &&
    timeout -k 10 300 python tools/config_bench.py $R >> $O/spec_tree_ab.jsonl &&
    IPMC_LIB_PATH=$V timeout -k 10 300 python tools/config_bench.py $R >> $O/spec_tree_ab.jsonl &&
    timeout -k 10 300 python tools/config_bench.py cfg2@16384 cfg4 ts6 >> $O/spec_tree_seq_ab.jsonl &&
    IPMC_LIB_PATH=$V timeout -k 10 300 python tools/config_bench.py cfg2@16384 cfg4 ts6 >> $O/spec_tree_seq_ab.jsonl
    ;;
  s7)
    # the reference's studies (examples/) with speculation trees against the
    # two-path build, 1 024 chains and one chain; the sequential Burgers /
    # two-scale sweeps again, interleaved
    V=ip_mcmc_amd/lib/variants/pathspec/libipmc.so
    for lib in "" "$V"; do
      tag=${lib:+pathspec}; tag=${tag:-tree}
      for args in "burgers_beta.py 1024" "burgers_beta.py 1" "lorenz_thesis.py 1024" "lorenz_thesis.py 1" "lorenz63_config2.py"; do
        set -- $args
        IPMC_LIB_PATH=$lib timeout -k 10 300 python examples/$1 ${2:-} > $O/ex_tmp.jsonl || exit 1
        python -c "import json,sys;[print(json.dumps(dict(json.loads(l),build='$tag',example='$1',arg='${2:-}'))) for l in open('$O/ex_tmp.jsonl') if l.startswith('{')]" >> $O/examples_tree_ab.jsonl || exit 1
      done
    done &&
    for i in 1 2; do
      timeout -k 10 300 python tools/config_bench.py cfg4 ts6 >> $O/seq_tree_ab2.jsonl &&
      IPMC_LIB_PATH=$V timeout -k 10 300 python tools/config_bench.py cfg4 ts6 >> $O/seq_tree_ab2.jsonl || exit 1
    done
    ;;
  s8)
    # speculation trees with the finer rate grid and 0.95 memory: speculative
    # parity tests, the small-ensemble rows and the studies against the
    # two-path build, then the whole suite
    V=ip_mcmc_amd/lib/variants/pathspec/libipmc.so
    timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
        -k "speculative or dense_prior or small_models" > $O/pytest_tree_spec2.log 2>&1 &&
    R="l96mx1@256 l96mx64@256 l96mx1024@256 l96x1@256 l96x64@256" &&
    timeout -k 10 300 python tools/config_bench.py $R cfg2@16384 >> $O/spec_tree_ab2.jsonl &&
    IPMC_LIB_PATH=$V timeout -k 10 300 python tools/config_bench.py $R cfg2@16384 >> $O/spec_tree_ab2.jsonl &&
    for lib in "" "$V"; do
      tag=${lib:+pathspec}; tag=${tag:-tree}
      for args in "burgers_beta.py 1024" "burgers_beta.py 1" "lorenz_thesis.py 1024" "lorenz_thesis.py 1"; do
        set -- $args
        IPMC_LIB_PATH=$lib timeout -k 10 300 python examples/$1 ${2:-} > $O/ex_tmp.jsonl || exit 1
        python -c "import json,sys;[print(json.dumps(dict(json.loads(l),build='$tag',example='$1',arg='${2:-}'))) for l in open('$O/ex_tmp.jsonl') if l.startswith('{')]" >> $O/examples_tree_ab2.jsonl || exit 1
      done
    done &&
    { timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_s8.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; }
    ;;
  s9)
    # Burgers small ensembles: trees vs two paths vs no speculation, CFL and fixed step
    V=ip_mcmc_amd/lib/variants/pathspec/libipmc.so
    P="python tools/probes/burgers_spec_probe.py"
    for i in 1 2; do
      timeout -k 10 200 $P 1024 >> $O/burgers_spec_probe.jsonl &&
      IPMC_LIB_PATH=$V timeout -k 10 200 $P 1024 >> $O/burgers_spec_probe.jsonl || exit 1
    done &&
    timeout -k 10 200 $P 1024 1 >> $O/burgers_spec_probe.jsonl &&
    timeout -k 10 200 $P 1 >> $O/burgers_spec_probe.jsonl &&
    IPMC_LIB_PATH=$V timeout -k 10 200 $P 1 >> $O/burgers_spec_probe.jsonl
    ;;
  s10)
    # estimator memory 3/4 (product) vs 0.95 vs the two paths: Burgers
    # studies (CFL and fixed step), the mixing rows, the Lorenz study
    P="python tools/probes/burgers_spec_probe.py"
    R="l96mx1@256 l96mx64@256 l96mx1024@256 cfg2@16384"
    for lib in "" ip_mcmc_amd/lib/variants/m095/libipmc.so ip_mcmc_amd/lib/variants/pathspec/libipmc.so; do
      IPMC_LIB_PATH=$lib timeout -k 10 200 $P 1024 >> $O/mem_ab_burgers.jsonl &&
      IPMC_LIB_PATH=$lib timeout -k 10 200 $P 1 >> $O/mem_ab_burgers.jsonl &&
      IPMC_LIB_PATH=$lib timeout -k 10 200 python tools/config_bench.py $R | \
        python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin]" >> $O/mem_ab_rows.jsonl &&
      IPMC_LIB_PATH=$lib timeout -k 10 200 python examples/lorenz_thesis.py 1024 | \
        python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin if l.startswith('{')]" >> $O/mem_ab_lorenz.jsonl || exit 1
    done
    ;;
  s11)
    # run-to-run spread of the Burgers pCN CFL study (1 024 chains), three builds interleaved
    P="python tools/probes/burgers_spec_probe.py"
    for i in 1 2 3; do
      for lib in "" ip_mcmc_amd/lib/variants/m095/libipmc.so ip_mcmc_amd/lib/variants/pathspec/libipmc.so; do
        IPMC_LIB_PATH=$lib timeout -k 10 200 $P 1024 0 pcn-cfl >> $O/burgers_pcn_cfl_spread.jsonl || exit 1
      done
    done
    ;;
  final)
    # the final tree: the whole suite, the published line with its same-box
    # profiles, the small-ensemble rows and the reference studies
    { timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_final.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; } &&
    bash tools/sessions/r4.sh s2prof &&
    timeout -k 10 300 python tools/config_bench.py l96mx1@256 l96mx64@256 l96mx1024@256 l96x1@256 l96x64@256 \
        cfg2@16384 > $O/spec_final.jsonl &&
    for args in "burgers_beta.py 1024" "burgers_beta.py 1" "lorenz_thesis.py 1024" "lorenz_thesis.py 1" \
                "lorenz63_config2.py" "stuart_reference.py"; do
      set -- $args
      timeout -k 10 300 python examples/$1 ${2:-} > $O/ex_tmp.jsonl || exit 1
      python -c "import json,sys;[print(json.dumps(dict(json.loads(l),example='$1',arg='${2:-}'))) for l in open('$O/ex_tmp.jsonl') if l.startswith('{')]" >> $O/examples_final.jsonl || exit 1
    done
    ;;
  s12b)
    # kernel trace of the Burgers pCN CFL study, 1 024 chains, auto speculation and none
    for sp in 0 1; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/burtrace$sp -o run -- \
          python tools/probes/burgers_spec_probe.py 1024 $sp pcn-cfl > $O/burtrace$sp.json || exit 1
    done
    ;;
  s13)
    # Burgers studies at 1 024 and 256 chains: speculation width 1 / 2 / 4 / auto, CFL and fixed step
    P="python tools/probes/burgers_spec_probe.py"
    for sp in 1 2 4 0; do
      timeout -k 10 200 $P 1024 $sp >> $O/burgers_width_scan.jsonl || exit 1
    done &&
    timeout -k 10 200 $P 256 1 >> $O/burgers_width_scan.jsonl &&
    timeout -k 10 200 $P 256 0 >> $O/burgers_width_scan.jsonl
    ;;
  s14)
    # config 2: the Lorenz-63 RK4 loop unrolled by 2 and 4 against the compiler's choice, interleaved
    for i in 1 2; do
      for lib in "" ip_mcmc_amd/lib/variants/l63u2/libipmc.so ip_mcmc_amd/lib/variants/l63u4/libipmc.so; do
        IPMC_LIB_PATH=$lib timeout -k 10 200 python tools/config_bench.py cfg2@16384 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin]" >> $O/l63_unroll_ab.jsonl || exit 1
      done
    done
    ;;
  s15)
    # the Lorenz-63 RK loop unrolled by 4 (product): its parity tests, the
    # unroll A/B (compiler's choice / 4 / 8), the config-2 study, the whole suite
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests \
        -m gpu -k "small or cfg2 or l63 or L63 or dense_prior or speculative" > $O/pytest_l63_unroll.log 2>&1 &&
    for i in 1 2; do
      for lib in ip_mcmc_amd/lib/variants/l63u0/libipmc.so "" ip_mcmc_amd/lib/variants/l63u8/libipmc.so; do
        IPMC_LIB_PATH=$lib timeout -k 10 200 python tools/config_bench.py cfg2@16384 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product_u4}'))) for l in sys.stdin]" >> $O/l63_unroll_ab2.jsonl || exit 1
      done
    done &&
    timeout -k 10 200 python examples/lorenz63_config2.py > $O/example_l63_cfg2.jsonl &&
    { timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_s15.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; }
    ;;
  s16)
    # the Lorenz-96 RK loop unrolled by 2 (variant) against the product: the
    # headline kernel leg and the small-ensemble rows, interleaved
    V=ip_mcmc_amd/lib/variants/l96u2/libipmc.so
    for i in 1 2; do
      for lib in "" "$V"; do
        IPMC_LIB_PATH=$lib timeout -k 10 300 python bench.py --kernel-only --no-cpu --steps 50 --warmup 5 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin if l.startswith('{')]" >> $O/l96_unroll_ab.jsonl &&
        IPMC_LIB_PATH=$lib timeout -k 10 300 python tools/config_bench.py l96mx1@256 l96mx64@256 l96mx1024@256 l96x64@256 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product}'))) for l in sys.stdin]" >> $O/l96_unroll_ab.jsonl || exit 1
      done
    done
    ;;
  final2)
    # the exact tree the round ends on: the suite, smoke(), the default bench line
    { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_final2.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ]; } &&
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final2.log 2>&1 &&
    timeout -k 10 600 python bench.py > $O/bench_default_final2.json 2> $O/bench_default_final2.err
    ;;
  s17)
    # config 1 on the device path (one chain, linear G) with speculation trees;
    # the Lorenz-63 loop unrolled by 8: its parity tests on the variant, then
    # config 2 against the product (4), interleaved
    V=ip_mcmc_amd/lib/variants/l63u8/libipmc.so
    timeout -k 10 300 python tools/probes/cfg1_e2e.py > $O/cfg1_e2e_final.jsonl &&
    IPMC_LIB_PATH=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests \
        -m gpu -k "small or cfg2 or l63 or L63 or dense_prior or speculative" > $O/pytest_l63u8.log 2>&1 &&
    for i in 1 2; do
      for lib in "" "$V"; do
        IPMC_LIB_PATH=$lib timeout -k 10 200 python tools/config_bench.py cfg2@16384 | \
          python -c "import json,sys;[print(json.dumps(dict(json.loads(l),lib='${lib:-product_u4}'))) for l in sys.stdin]" >> $O/l63_unroll_ab3.jsonl || exit 1
      done
    done
    ;;
  s18)
    # in-wave trees resolved in parallel (small_spec_kernel) and the Lorenz-63
    # loop unrolled by 8: the speculative parity tests, config 1 on the device
    # path, config 2, then the whole suite
    timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests \
        -m gpu -k "small or cfg2 or l63 or L63 or dense_prior or speculative or linear or sampler" > $O/pytest_s18_spec.log 2>&1 &&
    timeout -k 10 300 python tools/probes/cfg1_e2e.py > $O/cfg1_e2e_s18.jsonl &&
    timeout -k 10 200 python tools/config_bench.py cfg2@16384 > $O/cfg2_s18.jsonl &&
    timeout -k 10 200 python examples/lorenz63_config2.py > $O/example_l63_cfg2_s18.jsonl &&
    { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_s18.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ]; } &&
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_s18.log 2>&1
    ;;
  s19)
    # the small speculative kernel keeping its tree node across rounds
    timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests \
        -m gpu -k "small or cfg2 or l63 or L63 or dense_prior or speculative or linear or sampler" > $O/pytest_s19_spec.log 2>&1 &&
    timeout -k 10 300 python tools/probes/cfg1_e2e.py > $O/cfg1_e2e_s19.jsonl &&
    timeout -k 10 200 python tools/config_bench.py cfg2@16384 > $O/cfg2_s19.jsonl &&
    { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
        > $O/pytest_gpu_s19.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ]; } &&
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_s19.log 2>&1
    ;;
  s20)
    # config 2's SQ pass on the final kernel (unroll 8, parallel walk)
    SQS="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
    timeout -s KILL 90 rocprofv3 --pmc $SQS --kernel-trace --output-format csv -d $O/sq_cfg2_final/f64 -o run -- \
        python tools/config_bench.py cfg2@16384!f64 > /dev/null &&
    timeout -s KILL 90 rocprofv3 --pmc $SQS --kernel-trace --output-format csv -d $O/sq_cfg2_final/f32 -o run -- \
        python tools/config_bench.py cfg2@16384!f32 > /dev/null &&
    python tools/sq_summarize.py $O/sq_cfg2_final/f64 small_spec_kernel > $O/sq_cfg2_final_f64.json &&
    python tools/sq_summarize.py $O/sq_cfg2_final/f32 small_spec_kernel > $O/sq_cfg2_final_f32.json
    ;;
  dbg)
    timeout -k 10 300 python tools/probes/spec_tree_debug.py > $O/spec_tree_debug.txt 2>&1 &&
    IPMC_LIB_PATH=ip_mcmc_amd/lib/variants/burshfl/libipmc.so timeout -k 10 300 python tools/probes/spec_tree_debug.py \
        > $O/spec_tree_debug_shfl.txt 2>&1
    ;;
  *) echo "unknown session $1"; exit 2 ;;
esac
