#!/bin/bash
# Evidence for profiles/: default bench line, rocprofv3 kernel stats of the same
# workload, separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md recipe),
# a device-side step timeline (tools/trace_probe.py) and the 5000-wide aggregation
# probe's kernel stats + PMC traffic.  Run on the GPU box:
#   gpurun -- 'bash tools/profile_round.sh gpurun_out/prof_r02'
set -eo pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
ROOT=$(pwd)
LIGHT="--no-cpu-baseline --compare-dense 0 --compare-dropedge 0 --aggregation 0"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python bench.py $LIGHT > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -- \
  python bench.py $LIGHT --steps 5 --warmup 2 > /dev/null 2> "$OUT/fetch.log"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -- \
  python bench.py $LIGHT --steps 5 --warmup 2 > /dev/null 2> "$OUT/write.log"
python tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" --out "$OUT/pmc_traffic.json" > "$OUT/pmc_traffic.txt"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline" -o run -- \
  python tools/trace_probe.py --mode both > "$OUT/timeline.log" 2>&1
python tools/step_timeline.py "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 8 > "$OUT/timeline_step.txt"
python tools/step_timeline.py "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 20 > "$OUT/timeline_chain_alone.txt"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/agg" -o run -- \
  python tools/agg_probe.py > "$OUT/agg_probe.txt" 2> "$OUT/agg.log"
# HBM traffic of the 5000-wide aggregation (k_spmm_slice + fixup), TD and BU graphs apart
for g in td bu; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/agg_fetch_$g" -- \
    python tools/agg_probe.py --graphs $g --no-streams --iters 5 > /dev/null 2>> "$OUT/agg.log"
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/agg_write_$g" -- \
    python tools/agg_probe.py --graphs $g --no-streams --iters 5 > /dev/null 2>> "$OUT/agg.log"
  python tools/pmc_traffic.py "$OUT/agg_fetch_$g" "$OUT/agg_write_$g" --out "$OUT/agg_pmc_$g.json" \
    > "$OUT/agg_pmc_$g.txt"
done
echo done
