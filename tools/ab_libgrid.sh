#!/bin/bash
# A/B of library variants over workloads, interleaved reps (box-to-box and run-to-run
# noise shows up as spread):  WL="twitter15 weibo_bf16" bash tools/ab_libgrid.sh base build/variants/x.so ...
set -eo pipefail
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --steps 200 --warmup 10"
for rep in ${REPS:-1 2 3}; do
for v in "$@"; do
for w in ${WL:-twitter15}; do
  tag=$(basename "$v" .so)
  if [ "$v" = base ]; then unset BGCN_LIB; else export BGCN_LIB=$(pwd)/$v; fi
  timeout -k 10 120 python bench.py $L --workload $w 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $w', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done; done; done
