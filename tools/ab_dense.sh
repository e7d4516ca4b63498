#!/bin/bash
# Dense-path bench lines per library variant (BGCN_LIB), plus the pheme768 workload with the
# in-tree library:  gpurun -- 'bash tools/ab_dense.sh build/variants/libbgcn_a.so ...'
set -eo pipefail
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --dropin 0 --host-fed 0 --steps 40 --warmup 5"
for v in "$@"; do
  tag=$(basename "$v" .so)
  export BGCN_LIB=$(pwd)/$v
  timeout -k 10 200 python bench.py $L --feat-mode dense 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag dense', d['value'], d['ms_per_step'], json.dumps(d['kernels']))" >> gpurun_out/ab_dense.txt
done
unset BGCN_LIB
timeout -k 10 200 python bench.py $L --workload pheme768 > gpurun_out/pheme768.json 2>gpurun_out/pheme768.log
python -c "import json; d=json.load(open('gpurun_out/pheme768.json')); print('pheme768', d['value'], d['ms_per_step'], json.dumps(d['roofline']))" >> gpurun_out/ab_dense.txt
