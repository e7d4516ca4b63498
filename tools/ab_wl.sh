#!/bin/bash
# Interleaved A/B of library variants over the bench workloads (BGCN_LIB selects a
# variant; "cur" = the in-tree lib): ms per step, `rounds` passes.  On the GPU box:
#   bash tools/ab_wl.sh "twitter15 weibo_bf16" 2 cur build/variants/libbgcn_base.so
set -eo pipefail
WLS=$1; ROUNDS=$2; shift 2
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --dropin 0 --steps 100 --warmup 10"
OUT=gpurun_out/ab_wl.txt
for r in $(seq 1 "$ROUNDS"); do
  for wl in $WLS; do
    for v in "$@"; do
      if [ "$v" = cur ]; then unset BGCN_LIB; tag=cur; else export BGCN_LIB=$(pwd)/$v; tag=$(basename "$v" .so); fi
      timeout -k 10 150 python bench.py $L --workload "$wl" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $wl $tag', d['value'], d['ms_per_step'], d['invalid_steps'])" >> $OUT
    done
  done
done
cat $OUT
