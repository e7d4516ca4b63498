#!/bin/bash
# Evidence for profiles/ (round 6): per workload the bench line, rocprofv3 kernel stats of the
# same command and its per-launch-form table (tools/prof.py forms: the in-step X pass apart
# from the standalone ones), separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md
# recipe; tools/prof.py traffic) -> pmc_traffic_<workload>.json (bench.py's roofline.traffic
# reads profiles/r06_pmc_traffic_<workload>[_dense].json); the dense feature path's PMC
# traffic and SQ counters (twitter15 --feat-mode dense); the device-side step timelines; the
# 5000-wide aggregation probe with its PMC traffic; the FETCH_SIZE calibration probe.
#   gpurun -- 'bash tools/profile_round.sh gpurun_out/prof_r06 twitter15 weibo_bf16 synth1024_bf16'
#   PARTS=agg,fetch,timeline,dense to run only those parts (default: all)
set -eo pipefail
OUT=${1:-gpurun_out/prof}; shift
WLS=${@:-twitter15}
PARTS=${PARTS:-bench,dense,timeline,agg,fetch}
mkdir -p "$OUT"
ROOT=$(pwd)
LIGHT="--no-cpu-baseline --compare-dense 0 --compare-dropedge 0 --aggregation 0 --dropin 0 --host-fed 0 --eval-path 0"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
has() { [[ ",$PARTS," == *",$1,"* ]]; }
if has bench; then
for w in $WLS; do
  # the same command without the profiler first: the profiler slows the step (its span of the
  # pass then reads the perturbed step's), so both step times are kept side by side
  timeout -k 10 300 python bench.py --workload $w $LIGHT > "$OUT/bench_unprofiled_$w.json" 2> "$OUT/unprofiled_$w.log"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_$w" -o run -- \
    python bench.py --workload $w $LIGHT > "$OUT/bench_under_rocprof_$w.json" 2> "$OUT/stats_$w.log"
  python tools/prof.py forms "$OUT/stats_$w/run_kernel_trace.csv" > "$OUT/kernel_forms_$w.txt"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$w" -- \
    python bench.py --workload $w $LIGHT --steps 5 --warmup 2 > /dev/null 2> "$OUT/fetch_$w.log"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$w" -- \
    python bench.py --workload $w $LIGHT --steps 5 --warmup 2 > /dev/null 2> "$OUT/write_$w.log"
  python tools/prof.py traffic "$OUT/fetch_$w" "$OUT/write_$w" --out "$OUT/pmc_traffic_$w.json" > "$OUT/pmc_traffic_$w.txt"
  echo "$w done"
done
fi
if has dense; then
  D="--workload twitter15 --feat-mode dense $LIGHT --steps 5 --warmup 2"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_dense" -- \
    python bench.py $D > /dev/null 2> "$OUT/fetch_dense.log"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_dense" -- \
    python bench.py $D > /dev/null 2> "$OUT/write_dense.log"
  python tools/prof.py traffic "$OUT/fetch_dense" "$OUT/write_dense" --out "$OUT/pmc_traffic_twitter15_dense.json" \
    > "$OUT/pmc_traffic_twitter15_dense.txt"
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq_dense" -- \
    python bench.py $D > /dev/null 2> "$OUT/sq_dense.log"
  python tools/prof.py counters "$OUT/sq_dense" > "$OUT/sq_dense.txt"
  echo "dense done"
fi
if has timeline; then
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline" -o run -- \
    python tools/trace_probe.py --mode both > "$OUT/timeline.log" 2>&1
  python tools/prof.py timeline "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 8 > "$OUT/timeline_step.txt"
  python tools/prof.py timeline "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 20 > "$OUT/timeline_chain_alone.txt"
  echo "timeline done"
fi
if has agg; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/agg" -o run -- \
    python tools/agg_probe.py > "$OUT/agg_probe.txt" 2> "$OUT/agg.log"
  for g in td bu; do
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/agg_fetch_$g" -- \
      python tools/agg_probe.py --graphs $g --no-streams --iters 5 > /dev/null 2>> "$OUT/agg.log"
    timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/agg_write_$g" -- \
      python tools/agg_probe.py --graphs $g --no-streams --iters 5 > /dev/null 2>> "$OUT/agg.log"
    python tools/prof.py traffic "$OUT/agg_fetch_$g" "$OUT/agg_write_$g" --out "$OUT/agg_pmc_$g.json" \
      > "$OUT/agg_pmc_$g.txt"
  done
  echo "agg done"
fi
if has fetch; then
  timeout -k 10 120 python tools/fetch_probe.py > "$OUT/fetch_probe_times.json" 2> "$OUT/fetch_probe.log"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_probe" -- \
    python tools/fetch_probe.py --reps 2 > /dev/null 2>> "$OUT/fetch_probe.log"
  python tools/fetch_probe.py --pmc-dir "$OUT/fetch_probe" > "$OUT/fetch_probe_pmc.json"
  echo "fetch probe done"
fi
echo done
