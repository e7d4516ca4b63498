#!/bin/bash
# Evidence for profiles/ (round 5): per workload the bench line, rocprofv3 kernel stats of
# the same command, separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md recipe;
# tools/prof.py traffic applies the gfx950 corrections) -> pmc_traffic_<workload>.json (what
# bench.py's roofline.traffic reads from profiles/r04_pmc_traffic_<workload>.json), the
# device-side step timelines and the 5000-wide aggregation probe with its PMC traffic.
#   gpurun -- 'bash tools/profile_round.sh gpurun_out/prof_r05 twitter15 weibo_bf16 synth1024_bf16'
set -eo pipefail
OUT=${1:-gpurun_out/prof}; shift
WLS=${@:-twitter15}
mkdir -p "$OUT"
ROOT=$(pwd)
LIGHT="--no-cpu-baseline --compare-dense 0 --compare-dropedge 0 --aggregation 0 --dropin 0 --host-fed 0 --eval-path 0"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for w in $WLS; do
  # the same command without the profiler first: the profiler slows the step (its span of the
  # pass then reads the perturbed step's), so both step times are kept side by side
  timeout -k 10 300 python bench.py --workload $w $LIGHT > "$OUT/bench_unprofiled_$w.json" 2> "$OUT/unprofiled_$w.log"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_$w" -o run -- \
    python bench.py --workload $w $LIGHT > "$OUT/bench_under_rocprof_$w.json" 2> "$OUT/stats_$w.log"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$w" -- \
    python bench.py --workload $w $LIGHT --steps 5 --warmup 2 > /dev/null 2> "$OUT/fetch_$w.log"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$w" -- \
    python bench.py --workload $w $LIGHT --steps 5 --warmup 2 > /dev/null 2> "$OUT/write_$w.log"
  python tools/prof.py traffic "$OUT/fetch_$w" "$OUT/write_$w" --out "$OUT/pmc_traffic_$w.json" > "$OUT/pmc_traffic_$w.txt"
  echo "$w done"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline" -o run -- \
  python tools/trace_probe.py --mode both > "$OUT/timeline.log" 2>&1
python tools/prof.py timeline "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 8 > "$OUT/timeline_step.txt"
python tools/prof.py timeline "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 20 > "$OUT/timeline_chain_alone.txt"
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
echo done
