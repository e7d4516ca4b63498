#!/bin/bash
# A/B of runtime knobs (environment variables read by libbgcn): the default bench line
# (light: no CPU baseline / comparisons) per setting, interleaved.
#   gpurun -- 'bash tools/ab_env.sh "BGCN_COMPACT_GROUP=1" "BGCN_COMPACT_GROUP=0" ...'
set -eo pipefail
L="--no-cpu-baseline --compare-dense 0 --compare-dropedge 0 --aggregation 0 --dropin 0 --host-fed 0 --steps 200 --warmup 10 $BENCH_ARGS"
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py $L 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d.get('compaction_standalone') or {}
print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline']['frac'],
      (c.get('paced') or {}).get('frac'), (c.get('unpaced') or {}).get('frac'))" >> gpurun_out/ab_env.txt
done
