#!/bin/bash
# A/B of library variants built with different compile-time knobs (build/variants/*.so,
# BGCN_LIB selects one per run): chain-alone time + per-kernel stats (shape_probe, 128
# trees) and the default bench step, per variant.  Usage on the GPU box:
#   bash tools/ab_libs.sh base build/variants/libbgcn_c128.so ...   ("base" = in-tree lib)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --dropin 0 --host-fed 0 --steps 200 --warmup 10 $BENCH_ARGS"
for v in "$@"; do
  tag=$(basename "$v" .so)
  if [ "$v" = base ]; then unset BGCN_LIB; else export BGCN_LIB=$(pwd)/$v; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$tag -o run -- \
    python tools/shape_probe.py --only "mean 256" --steps 50 > gpurun_out/ab_$tag.chain.txt 2>&1
  timeout -k 10 120 python bench.py $L 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])" >> gpurun_out/ab_bench.txt
  grep chain gpurun_out/ab_$tag.chain.txt | sed "s/^/$tag /" >> gpurun_out/ab_bench.txt
done
