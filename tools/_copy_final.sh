#!/bin/bash
# copy the regenerated round-3 evidence from gpurun_out/final into profiles/
set -e
F=gpurun_out/final
P=profiles
cp $F/prof/bench.json $P/r03_bench.json
cp $F/prof/bench_under_rocprof.json $P/r03_bench_under_rocprof.json
cp $F/prof/stats/run_kernel_stats.csv $P/r03_kernel_stats.csv
cp $F/prof/pmc_traffic.json $P/r03_pmc_traffic.json
cp $F/prof/pmc_traffic.txt $P/r03_pmc_traffic.txt
cp $F/prof/timeline_step.txt $P/r03_timeline_step.txt
cp $F/prof/timeline_chain_alone.txt $P/r03_timeline_chain_alone.txt
cp $F/prof/agg_probe.txt $P/r03_aggregation_probe.txt
cp $F/prof/agg/run_kernel_stats.csv $P/r03_aggregation_kernel_stats.csv
cp $F/prof/agg_pmc_td.json $P/r03_agg_pmc_td.json
cp $F/prof/agg_pmc_bu.json $P/r03_agg_pmc_bu.json
cp $F/qb/weibo_bf16.json $P/r03_bench_weibo_bf16.json
cp $F/qb/synth1024_bf16.json $P/r03_bench_synth1024_bf16.json
cp $F/qb/twitter15_tail.json $P/r03_bench_twitter15_tail.json
cp $F/stats_weibo_bf16/run_kernel_stats.csv $P/r03_weibo_bf16_kernel_stats.csv
cp $F/stats_synth1024_bf16/run_kernel_stats.csv $P/r03_synth1024_bf16_kernel_stats.csv
cp $F/stats_twitter15_tail/run_kernel_stats.csv $P/r03_tail_kernel_stats.csv
cp $F/gpu_tests.log $P/r03_gpu_tests_final.log
echo copied
