#!/bin/bash
# Round 3 GPU session (tools/gpu_session.sh stops at the first fault/abort/time-out).
#   tools/sessions/r3.sh <name>   -- the steps of session <name>
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
PYT="python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -rf"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-extra"
case "$1" in
  a)  # host loop, FMA-vs-reference, full-size configs, bench plumbing; then everything
    tools/gpu_session.sh \
      "new_tests:600:$PYT -v -s tests/test_gpu_hostloop.py tests/test_gpu_arith_agreement.py tests/test_gpu_fullsize.py tests/test_gpu_bench_dist.py -m gpu" \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
      "bench:400:python bench.py > gpurun_out/bench_line.json" \
      "arith:400:python tools/arith_agreement.py 100 0.2 0.05 0.02 > gpurun_out/arith_agreement.jsonl" \
      "cfg2:300:python tools/config_bench.py cfg2@128 cfg2g1@128 cfg2 > gpurun_out/cfg2.jsonl" \
      "stuart:400:python examples/stuart_reference.py > gpurun_out/stuart_reference.jsonl"
    ;;
  k)  # L96 FMA arith with the forcing folded into the stage bases (18 instead of 20 FP64 ops per component-step)
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "bench:400:python bench.py > gpurun_out/bench_line_fold.json" \
      "configs:500:python tools/config_bench.py cfg5 l96x1@256 l96x64@256 l96x1024@64 l96x8192@8 > gpurun_out/configs_fold.jsonl" \
      "arith:600:python tools/arith_agreement.py 100 0.2 0.05 0.02 > gpurun_out/arith_agreement_fold.jsonl"
    ;;
  m)  # A/B: the folded-forcing L96 kernels against the previous ones (variants/oldl96), bench + SQ pass each
    O=ip_mcmc_amd/lib/variants/oldl96/libipmc.so
    BB="python bench.py --steps 100 --warmup 5 --no-cpu --no-extra"
    tools/gpu_session.sh \
      "ab1:300:$BB > gpurun_out/ab_new.jsonl && IPMC_LIB_PATH=$O $BB > gpurun_out/ab_old.jsonl" \
      "ab2:300:$BB >> gpurun_out/ab_new.jsonl && IPMC_LIB_PATH=$O $BB >> gpurun_out/ab_old.jsonl" \
      "f32:300:$BB --dtype f32 >> gpurun_out/ab_new.jsonl && IPMC_LIB_PATH=$O $BB --dtype f32 >> gpurun_out/ab_old.jsonl" \
      "lanes4:300:$BB --dtype f32 --lanes 4 >> gpurun_out/ab_new.jsonl && IPMC_LIB_PATH=$O $BB --dtype f32 --lanes 4 >> gpurun_out/ab_old.jsonl && $BB --lanes 4 >> gpurun_out/ab_new.jsonl && IPMC_LIB_PATH=$O $BB --lanes 4 >> gpurun_out/ab_old.jsonl" \
      "sq_new:200:timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_fold_new -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-extra" \
      "sq_old:200:IPMC_LIB_PATH=$O timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_fold_old -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-extra"
    ;;
  n)  # strong-scaled shards on the bench problem: 4 lanes per chain with 1 / 2 / 4 slots, 512-step launches
    cmds=""
    for c in 8192 16384; do for lw in "2 0" "4 1" "4 2" "4 4" "2 2" "2 4"; do set -- $lw
      cmds="$cmds python bench.py --chains $c --lanes $1 --spec-width $2 --steps-per-launch 512 --steps 1024 --warmup 512 --no-cpu --no-extra >> gpurun_out/bench_shards_l4.jsonl &&"
    done; done
    tools/gpu_session.sh "shards:900:${cmds} true"
    ;;
  o)  # the 8-GPU strong-scaled shard (8 192 chains) at short timed regions: K = 20 / 200 steps, layouts
    cmds=""
    for K in "20 5" "200 10"; do set -- $K; k=$1; w=$2
      for lw in "2 0" "2 4" "4 2" "4 4" "8 1" "4 1"; do set -- $lw
        cmds="$cmds python bench.py --chains 8192 --lanes $1 --spec-width $2 --steps $k --warmup $w --no-cpu --no-extra >> gpurun_out/bench_8192_short.jsonl &&"
      done
    done
    tools/gpu_session.sh "short:900:${cmds} true"
    ;;
  p)  # LPC 8 halos by DPP (row_shr/row_shl + select) instead of ds_bpermute: parity, then the 8 192-chain shard
    cmds=""
    for K in "20 5" "200 10"; do set -- $K; k=$1; w=$2
      for lw in "8 1" "4 2"; do set -- $lw
        cmds="$cmds python bench.py --chains 8192 --lanes $1 --spec-width $2 --steps $k --warmup $w --no-cpu --no-extra >> gpurun_out/bench_8192_l8dpp.jsonl &&"
      done
    done
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "short:600:${cmds} true" \
      "layouts:300:python tools/config_bench.py cfg5 l96x65536@1:8 > gpurun_out/configs_l8dpp.jsonl"
    ;;
  q)  # the LPC-8 interleaved layouts in the auto plan: parity, fp32 packed 8-lane layouts, the 8 192 shard
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "f32:400:python tools/config_bench.py 'l96x16384!f32' 'l96x16384:4^1!f32' 'l96d16x16384!f32' 'l96d16x16384:4^1!f32' 'l96d80x16384!f32' 'l96d80x16384:16^2!f32' > gpurun_out/layouts_l8il.jsonl" \
      "f64:400:python tools/config_bench.py 'l96x8192!f64' 'l96x8192@512!f64' 'l96x8192@512:8~1!f64' 'l96d80x16384!f64' 'l96d16x16384!f64' >> gpurun_out/layouts_l8il.jsonl" \
      "bench:600:python bench.py --chains 8192 --steps 20 --warmup 5 --no-cpu --no-extra > gpurun_out/bench_8192_auto.jsonl && python bench.py --chains 8192 --steps 200 --warmup 10 --no-cpu --no-extra >> gpurun_out/bench_8192_auto.jsonl && python bench.py --chains 8192 --steps 1024 --warmup 512 --no-cpu --no-extra >> gpurun_out/bench_8192_auto.jsonl && python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_65536_k20.jsonl"
    ;;
  r)  # short timed regions with the clock-settling pre-warm: N=1 and the N=8 shard, K = 20 / 200
    tools/gpu_session.sh \
      "bench:600:python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > gpurun_out/bench_settle.jsonl && python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --settle 0 >> gpurun_out/bench_settle.jsonl && python bench.py --chains 8192 --steps 20 --warmup 5 --no-cpu --no-extra >> gpurun_out/bench_settle.jsonl && python bench.py --chains 8192 --steps 200 --warmup 10 --no-cpu --no-extra >> gpurun_out/bench_settle.jsonl && python bench.py --chains 16384 --steps 20 --warmup 5 --no-cpu --no-extra >> gpurun_out/bench_settle.jsonl && python bench.py --chains 32768 --steps 20 --warmup 5 --no-cpu --no-extra >> gpurun_out/bench_settle.jsonl"
    ;;
  s)  # where MCMCSampler.run's end-to-end time goes: kernel + memory-copy trace of the e2e workload
    tools/gpu_session.sh \
      "e2e:300:python tools/sampler_e2e.py 65536 20 1 > gpurun_out/e2e_plain.jsonl" \
      "trace:300:timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/e2e_trace -o run -- python tools/sampler_e2e.py 65536 20 1"
    ;;
  t)  # e2e after the one-sample last copy block and a same-size warm-up; the bench line
    tools/gpu_session.sh \
      "e2e:300:python tools/sampler_e2e.py 65536 20 1 > gpurun_out/e2e_t.jsonl && python tools/sampler_e2e.py 65536 20 5 >> gpurun_out/e2e_t.jsonl" \
      "trace:300:timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2e_trace_t -o run -- python tools/sampler_e2e.py 65536 20 1" \
      "bench:400:python bench.py > gpurun_out/bench_line_t.json"
    ;;
  w)  # the parity suite, then e2e with page-locked H2D staging, its host profile and the bench line
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "e2e:300:python tools/sampler_e2e.py 65536 20 1 > gpurun_out/e2e_w.jsonl && python tools/probes/e2e_host_profile.py > gpurun_out/e2e_host_profile_w.txt" \
      "bench:400:python bench.py > gpurun_out/bench_line_w.json"
    ;;
  x)  # H2D staging probe
    tools/gpu_session.sh "h2d:200:python tools/probes/h2d_probe.py > gpurun_out/h2d_probe.txt"
    ;;
  bq)  # Burgers config 4 per-GPU share (2 048 chains): SQ pass and the layouts
    tools/gpu_session.sh \
      "sq:200:timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_cfg4 -o run -- python tools/config_bench.py cfg4" \
      "layouts:300:python tools/config_bench.py cfg4 cfg4:16 cfg4:64 cfg4visc cfg4cfl > gpurun_out/cfg4_layouts.jsonl"
    ;;
  bn)  # Burgers config 4 share at 250 / 500 / 1000 / 2000 time steps: the per-pCN-step overhead
    tools/gpu_session.sh "fit:300:python tools/config_bench.py cfg4n250 cfg4n500 cfg4n1000 cfg4n2000 > gpurun_out/cfg4_nsteps.jsonl"
    ;;
  y2)  # the 8-GPU shard under both plans vs the oracle
    tools/gpu_session.sh "shard:600:$PYT -v tests/test_gpu_fullsize.py -k strong_scaled -m gpu"
    ;;
  y)  # the interleaved 8-lane layout with box / RW regularizer / schedule, and the fuzz
    tools/gpu_session.sh "il8:600:$PYT -q tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k 'interleaved or fuzz or every_layout' -m gpu"
    ;;
  z)  # the reference's config-1 script through the host step (one-chain float loop)
    tools/gpu_session.sh "stuart:400:python examples/stuart_reference.py > gpurun_out/stuart_reference.jsonl"
    ;;
  u)  # host-side profile of MCMCSampler.run (e2e)
    tools/gpu_session.sh "prof:300:python tools/probes/e2e_host_profile.py 65536 20 1 moments > gpurun_out/e2e_host_profile_moments.txt && python tools/probes/e2e_host_profile.py 65536 20 1 samples > gpurun_out/e2e_host_profile_samples.txt"
    ;;
  b)  # accept-path speculation (small models) and the K=6 two-scale layouts (SPL 3 DPP pairs / 1 / 6)
    V=ip_mcmc_amd/lib/variants
    tools/gpu_session.sh \
      "spec_tests:600:$PYT -q tests/test_gpu_ts_layout.py tests/test_gpu_fuzz.py tests/test_gpu_run.py tests/test_gpu_parity.py -k 'speculative or ts_ or fuzz or run or sampler' -m gpu" \
      "cfg2:300:python tools/config_bench.py cfg2@128 cfg2g1@128 cfg2@512 > gpurun_out/cfg2_accept_mode.jsonl" \
      "ts6_spl3:300:python tools/config_bench.py ts6 ts6@8 ts36 > gpurun_out/ts6_layouts.jsonl" \
      "ts6_spl1:300:IPMC_LIB_PATH=$V/ts6spl1/libipmc.so python tools/config_bench.py ts6 ts6@8 >> gpurun_out/ts6_layouts.jsonl" \
      "ts6_spl6:300:IPMC_LIB_PATH=$V/ts6spl6/libipmc.so python tools/config_bench.py ts6 ts6@8 >> gpurun_out/ts6_layouts.jsonl" \
      "ts6_spl3b:300:python tools/config_bench.py ts6 >> gpurun_out/ts6_layouts.jsonl" \
      "sq_cfg2:200:timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_cfg2 -o run -- python tools/config_bench.py cfg2@128" \
      "sq_ts6:200:timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_ts6 -o run -- python tools/config_bench.py ts6" \
      "examples:300:python examples/lorenz_thesis.py > gpurun_out/example_lorenz_thesis.json && python examples/stuart_examples.py > gpurun_out/example_stuart.jsonl" \
      "pytest_gpu:900:$PYT tests -m gpu -q"
    ;;
  d)  # the fixed tests; strong-scaling shards: speculative layouts filling 1 vs 2 waves per SIMD
    tools/gpu_session.sh \
      "spec_tests:600:$PYT -q tests/test_gpu_run.py tests/test_gpu_parity.py -k 'speculative or run' -m gpu" \
      "shards:500:python tools/config_bench.py l96x65536 l96x32768@2 l96x32768@2:2~2 l96x16384@4 l96x16384@4:2~4 l96x16384@4:4~2 l96x8192@8 l96x8192@8:2~8 l96x8192@8:2~4 l96x8192@8:4~4 l96x8192@16:2~8 > gpurun_out/shards.jsonl" \
      "cfg2:300:python tools/config_bench.py cfg2@1024 cfg2@1024~32 cfg2@1024~8 > gpurun_out/cfg2_1024.jsonl" \
      "sq_cfg2:200:timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_cfg2_1024 -o run -- python tools/config_bench.py cfg2@1024"
    ;;
  e)  # accept-path speculation in every kernel family: the parity suite, configs and the reference studies
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "configs:500:python tools/config_bench.py cfg2@1024 cfg4 cfg4visc cfg4cfl cfg4full cfg5 ts6 ts36 l96x1@256 l96x64@256 l96x1024@64 l96x8192@8 > gpurun_out/configs.jsonl" \
      "examples:400:python examples/lorenz_thesis.py > gpurun_out/example_lorenz_thesis.json && python examples/burgers_beta.py > gpurun_out/example_burgers_beta.jsonl && python examples/stuart_examples.py > gpurun_out/example_stuart.jsonl"
    ;;
  f)  # shard speculation cap (two waves per SIMD), the parity suite, then the shard sizes again
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "shards:500:python tools/config_bench.py l96x65536 l96x32768@2 l96x16384@4 l96x8192@8 l96x4096@16 l96x2048@16 > gpurun_out/shards_rule.jsonl" \
      "bench8:300:python bench.py --chains 8192 --no-cpu > gpurun_out/bench_8192.json"
    ;;
  g)  # strong-scaled shards on the bench's own problem: steps per launch 1 / 2 / 4 / 8 / 16
    cmds=""
    for c in 32768 16384 8192; do for l in 1 2 4 8 16; do
      cmds="$cmds python bench.py --chains $c --steps-per-launch $l --steps 96 --warmup 16 --no-cpu --no-extra >> gpurun_out/bench_shards.jsonl &&"
    done; done
    tools/gpu_session.sh "shards:900:${cmds} true"
    ;;
  h)  # why speculative shards are slow on the bench problem: per-dispatch times, reject-only variant
    V=ip_mcmc_amd/lib/variants
    tools/gpu_session.sh \
      "trace:300:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace16k -o run -- python bench.py --chains 16384 --steps-per-launch 4 --steps 48 --warmup 8 --no-cpu --no-extra" \
      "rejonly:300:IPMC_LIB_PATH=$V/rejonly/libipmc.so python bench.py --chains 16384 --steps-per-launch 4 --steps 96 --warmup 16 --no-cpu --no-extra > gpurun_out/bench_rejonly.jsonl && IPMC_LIB_PATH=$V/rejonly/libipmc.so python bench.py --chains 8192 --steps-per-launch 8 --steps 96 --warmup 16 --no-cpu --no-extra >> gpurun_out/bench_rejonly.jsonl"
    ;;
  i)  # shards on the bench problem: long launches, slots per chain
    cmds=""
    for c in 16384 8192; do for l in 32 128; do for sw in 0 2 4 1; do
      cmds="$cmds python bench.py --chains $c --steps-per-launch $l --spec-width $sw --steps 256 --warmup 16 --no-cpu --no-extra >> gpurun_out/bench_shards_long.jsonl &&"
    done; done; done
    tools/gpu_session.sh "shards:1000:${cmds} true"
    ;;
  v)  # validation of the tree as committed: the whole GPU suite (verbose), smoke, the default bench line
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -v" \
      "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
      "bench:400:python bench.py > gpurun_out/bench_line.json"
    ;;
  c)  # the published line and its profiles from one box: bench, rocprofv3 --stats of the same
      # command, the three PMC passes (HBM bytes, clock, VALU issue) of the headline kernel
    tools/gpu_session.sh \
      "bench:400:python bench.py > gpurun_out/bench_line.json" \
      "stats:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python bench.py --no-cpu" \
      "fetch64:200:timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/fetch -o run -- $B" \
      "write64:200:timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc64/write -o run -- $B" \
      "sq64:200:timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc64/sq -o run -- $B" \
      "fetch32:200:timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/fetch -o run -- $B --dtype f32" \
      "write32:200:timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc32/write -o run -- $B --dtype f32" \
      "sq32:200:timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc32/sq -o run -- $B --dtype f32" \
      "summ:60:python tools/pmc_summarize.py gpurun_out/pmc64 f64 65536 gpurun_out/pmc_l96_f64.json && python tools/pmc_summarize.py gpurun_out/pmc32 f32 65536 gpurun_out/pmc_l96_f32.json" \
      "shards:600:for c in 32768 16384 8192; do python bench.py --chains \$c --steps 20 --warmup 5 --no-cpu --no-extra >> gpurun_out/bench_shards_k20.jsonl || exit 3; done" \
      "bench_strong:600:python bench.py --chains 16384 --no-cpu > gpurun_out/bench_16384.json && python bench.py --chains 8192 --no-cpu > gpurun_out/bench_8192.json"
    ;;
  ll)  # launch length vs the slowest chain: speculative ensembles at 1 024 / 4 096 / 16 384 steps per launch
    tools/gpu_session.sh \
      "cfg2:400:python tools/config_bench.py cfg2@1024 cfg2@4096 cfg2@16384 > gpurun_out/launch_len.jsonl" \
      "l96:400:python tools/config_bench.py 'l96x1024@1024!f64' 'l96x1024@8192!f64' 'l96x64@1024!f64' 'l96x64@8192!f64' >> gpurun_out/launch_len.jsonl"
    ;;
  lm)  # the sampler at 16 384 steps per launch: the long-launch test, the reference studies through run()
    tools/gpu_session.sh \
      "tests:600:$PYT -v tests/test_gpu_fullsize.py tests/test_gpu_run.py -k 'cfg2 or run or interval' -m gpu" \
      "examples:500:python examples/lorenz_thesis.py > gpurun_out/example_lorenz_thesis.json && python examples/burgers_beta.py > gpurun_out/example_burgers_beta.jsonl && python examples/stuart_examples.py > gpurun_out/example_stuart.jsonl"
    ;;
  sg)  # speculation guess over recent rounds (SpecGuess) vs the whole launch's ratio (variants/cum)
    V=ip_mcmc_amd/lib/variants/cum/libipmc.so
    tools/gpu_session.sh \
      "tests:600:$PYT -q tests/test_gpu_fullsize.py tests/test_gpu_run.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_ts_layout.py -k 'cfg2 or run or interval or fuzz or speculative or ts_' -m gpu" \
      "ex_new:300:python examples/burgers_beta.py > gpurun_out/guess_burgers_new.jsonl && python examples/lorenz_thesis.py > gpurun_out/guess_thesis_new.json" \
      "ex_cum:300:IPMC_LIB_PATH=$V python examples/burgers_beta.py > gpurun_out/guess_burgers_cum.jsonl && IPMC_LIB_PATH=$V python examples/lorenz_thesis.py > gpurun_out/guess_thesis_cum.json" \
      "cfg2:300:python tools/config_bench.py cfg2@16384 cfg2@1024 > gpurun_out/guess_cfg2_new.jsonl && IPMC_LIB_PATH=$V python tools/config_bench.py cfg2@16384 cfg2@1024 > gpurun_out/guess_cfg2_cum.jsonl"
    ;;
  c2)  # config 2 through MCMCSampler.run; a 65 536-step launch (the slowest-chain bound)
    tools/gpu_session.sh \
      "example:300:python examples/lorenz63_config2.py > gpurun_out/example_lorenz63_config2.jsonl" \
      "cfg2:300:python tools/config_bench.py cfg2@16384 cfg2@65536 > gpurun_out/launch_len_65536.jsonl"
    ;;
  ps)  # page-locked asynchronous copy of the final chain state: the suite, e2e, the bench line
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q" \
      "e2e:300:python tools/sampler_e2e.py 65536 20 1 > gpurun_out/e2e_ps.jsonl" \
      "bench:400:python bench.py > gpurun_out/bench_line_ps.json"
    ;;
  sk)  # the 8 192-chain shard at K = 20 vs 200: per-dispatch kernel times
    tools/gpu_session.sh \
      "k20:200:timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/shard_k20 -o run -- python bench.py --chains 8192 --steps 20 --warmup 5 --no-cpu --no-extra" \
      "k200:200:timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/shard_k200 -o run -- python bench.py --chains 8192 --steps 200 --warmup 10 --no-cpu --no-extra"
    ;;
  fc)  # final-tree config table (every config on one box)
    tools/gpu_session.sh \
      "configs:600:python tools/config_bench.py cfg2@16384 cfg4 cfg4visc cfg4cfl cfg4full cfg5 ts6 ts36 l96x1@256 l96x64@256 l96x1024@64 l96x8192@8 > gpurun_out/configs_final.jsonl"
    ;;
  rs)  # round sums in registers: the suite, run() moments on config 2, tolerance z's
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q -s" \
      "example:300:python examples/lorenz63_config2.py > gpurun_out/example_lorenz63_config2.jsonl" \
      "e2e:300:python tools/sampler_e2e.py 65536 20 1 > gpurun_out/e2e_rs.jsonl"
    ;;
  fin)  # final tree: the suite, smoke, e2e, then the published line and its same-box profiles (session c)
    tools/gpu_session.sh \
      "pytest_gpu:900:$PYT tests -m gpu -q -s" \
      "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
      "e2e:300:python tools/sampler_e2e.py 65536 20 1 > gpurun_out/e2e_final.jsonl" && tools/sessions/r3.sh c
    ;;
  ex)  # the reference studies on the final tree
    tools/gpu_session.sh \
      "examples:500:python examples/lorenz_thesis.py > gpurun_out/example_lorenz_thesis.json && python examples/burgers_beta.py > gpurun_out/example_burgers_beta.jsonl && python examples/stuart_examples.py > gpurun_out/example_stuart.jsonl && python examples/stuart_reference.py > gpurun_out/stuart_reference.jsonl"
    ;;
  *) echo "unknown session $1"; exit 2 ;;
esac
