#!/bin/bash
# Round-end evidence beside tools/profile_round.sh: optionally the GPU tests, the device-side
# step / chain timelines, the full default bench line (every comparison leg) and the light
# bench line of the other workloads.
#   gpurun -- 'bash tools/round_bench.sh gpurun_out/prof_r04 [tests]'
set -eo pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
if [ "${2:-}" = tests ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -2 "$OUT/gpu_tests.log"
fi
LIGHT="--no-cpu-baseline --compare-dense 0 --compare-dropedge 0 --aggregation 0 --dropin 0 --host-fed 0 --eval-path 0"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline" -o run -- \
  python tools/trace_probe.py --mode both > "$OUT/timeline.log" 2>&1
python tools/prof.py timeline "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 8 > "$OUT/timeline_step.txt"
python tools/prof.py timeline "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 20 > "$OUT/timeline_chain_alone.txt"
timeout -k 10 400 python bench.py > "$OUT/bench_full.json" 2> "$OUT/bench_full.log"
echo "full bench done"
for w in ${WORKLOADS:-weibo_bf16 synth1024_bf16 pheme768 twitter15_tail}; do
  timeout -k 10 200 python bench.py --workload "$w" $LIGHT > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.log"
  echo "$w done"
done
python - "$OUT" <<'EOF'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    d = json.load(open(f))
    r = d["roofline"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], r.get("avg_ms"), r.get("frac"), r.get("traffic"))
EOF
