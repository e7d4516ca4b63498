#!/bin/bash
# A/B runner for the environment overrides the kernels read per call: runs the spmm
# parity tests once, then the aggregation probe (or the step span probe) once per value.
#   gpurun -- 'AB_VAR=BGCN_SPMM_PLAN AB_VALUES="0 1" bash tools/agg_ab.sh'
#   gpurun -- 'AB_VAR=BGCN_DW1_SPLIT AB_VALUES="1 4" AB_PROBE="tools/span_probe.py --workload weibo_bf16" bash tools/agg_ab.sh'
# Overrides read today: BGCN_SPMM_PLAN (planned / merge-path aggregation),
# BGCN_DW1_SPLIT (waves per dW1 column), BGCN_PREP_BLOCKS (compaction grid cap).
set -eo pipefail
: "${AB_VAR:?set AB_VAR to the environment variable to vary}"
: "${AB_VALUES:?set AB_VALUES to the space-separated values}"
PROBE=${AB_PROBE:-tools/agg_probe.py}
OUT=${AB_OUT:-gpurun_out/agg_ab.txt}
mkdir -p "$(dirname "$OUT")"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 \
  --timeout-method thread -k spmm > "$(dirname "$OUT")/spmm_tests.log" 2>&1
for v in $AB_VALUES; do
  echo "== $AB_VAR=$v" >> "$OUT"
  env "$AB_VAR=$v" timeout -k 10 180 python $PROBE >> "$OUT" 2>&1
done
