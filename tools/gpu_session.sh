#!/bin/bash
# The one GPU-session runner: each named step runs under its own time limit with its log in
# gpurun_out/<tag>/; the first failing step ends the session (no retries, nothing after a fault).
#
# usage: tools/gpu_session.sh <tag> <step>...
#   tests[=file,file...]  pytest -m gpu (default: the whole tests/ directory)
#   smoke                 __graft_entry__.smoke()
#   bench                 python bench.py $BENCH_ARGS (the driver's default line, CPU baseline included)
#   trace                 rocprofv3 --kernel-trace --stats of a short bench (kernel stats CSV)
#   pmc-hop               rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / TCC hit+miss) of tools/micro_prop.py
#   pmc-bench             rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / TCC hit+miss) of a short bench
#                         with one target update per hop (GDD_PROP_PAIR=0: every k_hop launch is the
#                         roofline's unpaired hop); summarise with tools/pmc_summary.py <dir>/pmcb ...
#   lookahead-ab          bench.py (no CPU baseline) with GDD_MB_LOOKAHEAD = 1, 2, 3, 1, 2, 3
#   pmc-products          rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / TCC hit+miss) of tools/micro_prop.py
#                         products, the default hop and the 4-slice form (GDD_HOP_LANES=8)
#   phases                tools/phase_times.py (per-phase wall times of the bench step)
#   kernarg-ab            micro_kpp arxiv + bench: default / HIP_FORCE_DEV_KERNARG=1 / kernarg-preload build / both, twice
#   reassign-ab           bench.py with GDD_MB_REASSIGN_FORM = 0 / 3 (the r04 reassignment vs block shuffle + parallel copies), twice
#   reassign-trace        rocprofv3 kernel trace of a short bench at GDD_MB_REASSIGN_FORM = 0..3 + k_mb_reassign durations
#   reassign-stamps       tools/stamps.py (STAMPS=1 build) at GDD_MB_REASSIGN_FORM = 0..3
#   stop-ab               bench.py: stop word loaded with trip 1 (default) vs tested alone at entry (libgdd_stopentry.so), twice
#   kpp                   tools/micro_kpp.py (k-means++ round micro-benchmark)
#   spec-ab               k-means++ folds with / without the speculative searches (micro + bench, twice)
#   lloyd-small           tools/micro_lloyd_small.py (recsys KMeans: one-workgroup update / grouping on and off)
#   stamps-kpp            tools/stamps.py (MiniBatch step + k-means++ pair launch stamps), speculative searches off / on
#   kpp-big               tools/micro_kpp.py big (one workgroup per trial vs per-block rounds) + in-kernel stamps
#   inertia               tools/micro_inertia.py (parallel exact inertia vs the one-lane fold)
#   gap                   tools/probe/gap_probe (dependent launches: stream vs hipGraph replay)
#   graph-ab              tools/micro_graph.py (MiniBatchKMeans / k-means++ fits, eager vs graph replay)
#   inertia-ab            bench.py (no CPU baseline) with the parallel inertia vs the one-lane fold, twice each
#   chunk-ab              bench.py (no CPU baseline) with GDD_MB_CHUNK = 16, 8, 4 x GDD_MB_LOOKAHEAD = 1, 2, twice
#   fold-cols             tools/micro_fold_cols.py (products M-step over all columns vs one rank's slice)
#   capture-probe         tools/probe_capture_h2d.py (what a graph-captured pageable H2D copy reads at replay)
#   assign                tools/bench_assign.py (full assignment pass, fp32 vs bf16, three shapes)
#   assign-ab             tools/bench_assign.py with the wave-tile fp32 pass vs GDD_ASSIGN_PERSIST=1
#   hop-lanes             tools/micro_prop.py at arxiv / products with the XCD slice A/B switch
#   prop-pair             tools/micro_prop.py at arxiv / products, paired target updates on / off
#   reddit | products     tools/bench_induct.py | tools/bench_products.py (config 3 / 5 shapes)
#   recsys | alidisplay   tools/bench_recsys_e2e.py [alidisplay] (config 4 end to end)
#   products-lloyd        tools/prof_products_lloyd.py under rocprofv3 --kernel-trace --stats (the products
#                         record's KMeans, per-kernel split + final cluster sizes)
#   pad-ab                tools/prof_products_lloyd.py with the fold's padded copy on / off (GDD_FOLD_PAD), 3x
#   agent                 the transductive drop-in on synthetic ogbn-arxiv (main_transduct.sh's r=0.5% line)
# e.g. /usr/local/graft/bin/gpurun -- 'bash tools/gpu_session.sh r03a tests=tests/test_gpu_kpp.py bench trace'
set -o pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"

run() {  # run <limit-seconds> <log-name> <command...>
  local lim=$1 log=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$log.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $log failed (rc $rc)"
    tail -60 "$OUT/$log.log"
    exit $rc
  fi
  tail -2 "$OUT/$log.log" | cut -c1-400
}

for step in "$@"; do
  case "$step" in
    tests) run 1500 pytest_gpu $PYT tests ;;
    tests=*) run 1500 pytest_part $PYT $(echo "${step#tests=}" | tr ',' ' ') ;;
    smoke) run 300 smoke python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 600 bench python bench.py ${BENCH_ARGS} ;;
    trace) run 420 trace rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
             -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra ;;
    pmc-hop)
      run 120 pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o hop -- python3 tools/micro_prop.py
      run 120 pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o hop -- python3 tools/micro_prop.py
      run 120 pmc_hit rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_hit" -o hop -- python3 tools/micro_prop.py ;;
    pmc-bench)
      B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra"
      run 240 pmcb_fetch env GDD_PROP_PAIR=0 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcb/pmc_fetch" -o bench -- $B
      run 240 pmcb_write env GDD_PROP_PAIR=0 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcb/pmc_write" -o bench -- $B
      run 240 pmcb_hit env GDD_PROP_PAIR=0 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmcb/pmc_hit" -o bench -- $B ;;
    lookahead-ab) run 900 lookahead_ab bash -c 'for la in 1 2 3 1 2 3; do echo "lookahead $la"; GDD_MB_LOOKAHEAD=$la python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    chunk-ab) run 900 chunk_ab bash -c 'for c in 16 8 4 16 8 4; do for la in 1 2; do echo "chunk $c lookahead $la"; GDD_MB_CHUNK=$c GDD_MB_LOOKAHEAD=$la python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done; done' ;;
    pmc-products)
      for form in default lanes8; do
        E="GDD_PROP_PAIR=0"; [ "$form" = lanes8 ] && E="GDD_PROP_PAIR=0 GDD_HOP_LANES=8"
        run 300 pmcp_${form}_fetch env $E rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcp_$form/pmc_fetch" -o hop -- python3 tools/micro_prop.py products
        run 300 pmcp_${form}_write env $E rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcp_$form/pmc_write" -o hop -- python3 tools/micro_prop.py products
        run 300 pmcp_${form}_hit env $E rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmcp_$form/pmc_hit" -o hop -- python3 tools/micro_prop.py products
      done ;;
    pmc-prod)  # the products hop's counters, default form only (three separate passes)
      E="GDD_PROP_PAIR=0"
      run 300 pmcp_fetch env $E rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcp/pmc_fetch" -o hop -- python3 tools/micro_prop.py products
      run 300 pmcp_write env $E rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcp/pmc_write" -o hop -- python3 tools/micro_prop.py products
      run 300 pmcp_hit env $E rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmcp/pmc_hit" -o hop -- python3 tools/micro_prop.py products ;;
    phases) run 300 phases python tools/phase_times.py ;;
    kpp) run 300 kpp python tools/micro_kpp.py ;;
    kpp-par) run 300 kpp_par python tools/micro_kpp.py par ;;
    relabel) run 600 relabel python tools/micro_relabel.py ;;
    par-ab) run 900 par_ab bash -c 'for v in 0 1 0 1; do echo "GDD_KPP_PAR_CHAIN=$v"; GDD_KPP_PAR_CHAIN=$v python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    kernarg-ab) run 1000 kernarg_ab bash -c 'P=graph-distillation-for-recommendation_amd/gdd/lib/libgdd_preload.so; for r in ${KARG_REPS:-1}; do for v in base devkarg preload both; do echo "variant $v"; case $v in base) E="";; devkarg) E="HIP_FORCE_DEV_KERNARG=1";; preload) E="GDD_LIB_PATH=$P";; both) E="HIP_FORCE_DEV_KERNARG=1 GDD_LIB_PATH=$P";; esac; env $E python tools/micro_kpp.py arxiv || exit 1; env $E python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done; done' ;;
    reassign-ab) run 900 reassign_ab bash -c 'for v in 0 2 0 2; do echo "GDD_MB_REASSIGN_FORM=$v"; GDD_MB_REASSIGN_FORM=$v python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    reassign-trace)
      for v in 0 1 2 3; do
        run 420 reassign_trace$v env GDD_MB_REASSIGN_FORM=$v rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rtrace$v" -o bench \
             -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra || exit 1
        echo "form $v"; python3 tools/kernel_durations.py "$OUT/rtrace$v/bench_kernel_trace.csv" k_mb_reassign 24
      done ;;
    reassign-stamps) run 300 reassign_stamps bash -c 'for v in 0 1 2 3; do echo "GDD_MB_REASSIGN_FORM=$v"; GDD_MB_REASSIGN_FORM=$v python tools/stamps.py || exit 1; done' ;;
    stop-ab) run 900 stop_ab bash -c 'P=graph-distillation-for-recommendation_amd/gdd/lib/libgdd_stopentry.so; for v in hoisted entry hoisted entry; do echo "variant $v"; if [ $v = entry ]; then E="GDD_LIB_PATH=$P"; else E=""; fi; env $E python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    near-ab) run 900 near_ab bash -c 'for v in 0 3 6 0 3 6; do echo "GDD_MB_NEAR_STOP=$v"; GDD_MB_NEAR_STOP=$v python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    spec-ab) run 900 spec_ab bash -c 'python tools/micro_kpp.py spec && for v in 1 0 1 0; do echo "GDD_KPP_SPEC_SEARCH=$v"; export GDD_KPP_SPEC_SEARCH=$v; python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    lloyd-small) run 300 lloyd_small python tools/micro_lloyd_small.py ;;
    stamps-kpp) run 300 stamps_kpp bash -c 'GDD_KPP_SPEC_SEARCH=0 python tools/stamps.py && GDD_KPP_SPEC_SEARCH=1 python tools/stamps.py' ;;
    spec8-ab) run 600 spec8_ab bash -c 'for v in 0 1 0 1; do echo "GDD_KPP_SPEC_SEARCH=$v"; GDD_KPP_SPEC_SEARCH=$v python tools/micro_kpp.py one || exit 1; done; for v in 0 1 0 1; do echo "GDD_KPP_SPEC_SEARCH=$v"; GDD_KPP_SPEC_SEARCH=$v python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    bigspec-ab) run 600 bigspec_ab bash -c 'for v in 0 1 0 1; do echo "GDD_KPP_SPEC_SEARCH=$v"; GDD_KPP_SPEC_SEARCH=$v python tools/micro_kpp.py big || exit 1; done && python tools/stamps.py kpp-big' ;;
    kpp-big) run 300 kpp_big bash -c 'python tools/micro_kpp.py big && python tools/stamps.py kpp-big' ;;
    inertia) run 300 inertia bash -c 'python tools/micro_inertia.py && GDD_INERTIA_SEQ=1 python tools/micro_inertia.py' ;;
    gap) run 60 gap ./tools/probe/gap_probe ;;
    graph-ab) run 300 graph_ab python tools/micro_graph.py ;;
    fold-cols) run 300 fold_cols python tools/micro_fold_cols.py ;;
    capture-probe) run 120 capture_probe python tools/probe_capture_h2d.py ;;
    inertia-ab) run 600 inertia_ab bash -c 'for v in 0 1 0 1; do echo "GDD_INERTIA_SEQ=$v"; GDD_INERTIA_SEQ=$v python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 || exit 1; done' ;;
    kpp-products) run 300 kpp_products python tools/micro_kpp_products.py ;;
    assign) run 300 assign python tools/bench_assign.py ;;
    assign-ab) run 400 assign_ab bash -c 'python tools/bench_assign.py && GDD_ASSIGN_PERSIST=1 python tools/bench_assign.py && python tools/bench_assign.py' ;;
    hop-lanes) run 300 hop_lanes bash -c 'python tools/micro_prop.py && GDD_HOP_LANES=8 python tools/micro_prop.py && GDD_HOP_LANES=32 python tools/micro_prop.py && python tools/micro_prop.py products && GDD_HOP_LANES=8 python tools/micro_prop.py products' ;;
    prop-pair) run 300 prop_pair bash -c 'python tools/micro_prop.py && GDD_PROP_PAIR=0 python tools/micro_prop.py && python tools/micro_prop.py && GDD_PROP_PAIR=0 python tools/micro_prop.py && python tools/micro_prop.py products && GDD_PROP_PAIR=0 python tools/micro_prop.py products' ;;
    reddit) run 400 reddit python tools/bench_induct.py ;;
    products) run 600 products python tools/bench_products.py ;;
    pad-ab) run 400 pad_ab env PADS=${PADS:-11,10,11,10,11,10} python tools/prof_products_lloyd.py "$OUT/cluster_sizes.npy" ;;
    products-lloyd) run 400 products_lloyd rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/lloyd" -o lloyd -- python3 tools/prof_products_lloyd.py "$OUT/cluster_sizes.npy" ;;
    recsys) run 400 recsys python tools/bench_recsys_e2e.py ;;
    alidisplay) run 400 alidisplay python tools/bench_recsys_e2e.py alidisplay ;;
    agent) run 600 agent env PYTHONPATH=graph-distillation-for-recommendation_amd python -m gdd.train_clustgdd_transduct \
             --gpu_id 0 --dataset ogbn-arxiv --reduction_rate 0.005 --prop_num 18 --postprop_num 10 --alpha 0.91 \
             --predropout 0.6 --sp_ratio 0.1 --preep 1000 --postep 1000 --frcoe 1.9 --predcoe 0.025 --save 1 \
             --json "$OUT/agent_arxiv.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done"
