# A/B of a per-call library knob: bash tools/ab_env.sh VAR "v1 v2 ..." [workloads]
set -e
VAR=$1; VALS=$2; WL=${3:-twitter15}
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --steps 200 --warmup 10"
for rep in 1 2; do
for v in $VALS; do
for w in $WL; do
  env $VAR=$v timeout -k 10 120 python bench.py $L --workload $w 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v $w', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done; done; done
