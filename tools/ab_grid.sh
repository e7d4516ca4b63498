# A/B over combinations of knob settings: bash tools/ab_grid.sh "A=1 B=2" "A=3" ... (each arg one config)
set -e
L="--no-cpu-baseline --compare-dense 0 --aggregation 0 --compare-dropedge 0 --steps 200 --warmup 10"
WL=${WL:-twitter15}
for rep in 1 2; do
for cfg in "$@"; do
for w in $WL; do
  env $cfg timeout -k 10 120 python bench.py $L --workload $w 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $w', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done; done; done
