#!/bin/bash
# Device-side step timelines (chain alone + full step) for one workload:
#   gpurun -- 'bash tools/timeline_wl.sh gpurun_out/tl weibo_bf16'
set -eo pipefail
OUT=${1:-gpurun_out/tl}
WL=${2:-twitter15}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline_$WL" -o run -- \
  python tools/trace_probe.py --mode both --workload "$WL" > "$OUT/timeline_$WL.log" 2>&1
python tools/step_timeline.py "$OUT"/timeline_$WL/run_kernel_trace.csv --after k_alu --step 8 > "$OUT/step_$WL.txt"
python tools/step_timeline.py "$OUT"/timeline_$WL/run_kernel_trace.csv --after k_alu --step 20 > "$OUT/alone_$WL.txt"
cat "$OUT/alone_$WL.txt" "$OUT/step_$WL.txt"
