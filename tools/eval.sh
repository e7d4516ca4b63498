#!/bin/bash
# One GPU call: GPU tests, quick bench lines and the device-side step timelines.
#   gpurun -- 'bash tools/eval.sh gpurun_out/e1 [tests]'
set -eo pipefail
OUT=${1:-gpurun_out/eval}
mkdir -p "$OUT"
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -2 "$OUT/gpu_tests.log"
fi
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --steps 200 --warmup 10"
for w in ${WORKLOADS:-twitter15 weibo_bf16 synth1024_bf16}; do
  for r in 1 2; do
    timeout -k 10 120 python bench.py $L --workload $w 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])" | tee -a "$OUT/bench.txt"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline" -o run -- \
  python tools/trace_probe.py --mode both > "$OUT/timeline.log" 2>&1
python tools/step_timeline.py "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 8 > "$OUT/timeline_step.txt"
python tools/step_timeline.py "$OUT"/timeline/run_kernel_trace.csv --after k_alu --step 20 > "$OUT/timeline_chain_alone.txt"
cat "$OUT/timeline_chain_alone.txt" "$OUT/timeline_step.txt"
