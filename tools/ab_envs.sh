# A/B of combinations of per-call library knobs, each run twice:
#   bash tools/ab_envs.sh "A=1,B=0" "A=0" ... [-- workloads]
set -e
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --steps 200 --warmup 10"
WL=${WORKLOADS:-twitter15}
for rep in 1 2; do
for combo in "$@"; do
for w in $WL; do
  envs=$(echo "$combo" | tr ',' ' ')
  env $envs timeout -k 10 120 python bench.py $L --workload $w 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$combo $w', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done; done; done
