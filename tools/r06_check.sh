#!/bin/bash
# Round-6 GPU check: the GPU suite, then the driver's own bench command.
#   gpurun -- 'bash tools/r06_check.sh gpurun_out/r06a'
set -eo pipefail
OUT=${1:-gpurun_out/r06}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.log"
echo "bench done"
