#!/bin/bash
# Light bench lines (no CPU baseline / comparisons) for a list of workloads, one JSON
# line each under $OUT:  gpurun -- 'bash tools/quick_bench.sh gpurun_out/qb twitter15 weibo_bf16'
set -eo pipefail
OUT=$1; shift
mkdir -p "$OUT"
LIGHT="--no-cpu-baseline --compare-dense 0 --compare-dropedge 0 --aggregation 0 --dropin 0"
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload "$w" $LIGHT $BENCH_ARGS > "$OUT/$w.json" 2> "$OUT/$w.log"
  python -c "import json,sys; d=json.load(open('$OUT/$w.json')); print('$w', d['value'], d['ms_per_step'], d.get('invalid_steps'))"
done
