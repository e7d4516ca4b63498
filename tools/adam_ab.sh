set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/adam_ab
for v in ${VARIANTS:-img_r16c256}; do
  for mode in plain images; do
    export BGCN_LIB=$(pwd)/build/variants/libbgcn_$v.so
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/adam_ab/${v}_$mode -o run -- python tools/adam_probe.py $mode 300 > gpurun_out/adam_ab/${v}_$mode.log 2>&1
    f=$(ls gpurun_out/adam_ab/${v}_$mode/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/adam_ab/${v}_$mode/run_kernel_stats.csv)
    echo "$v $mode $(grep k_adam $f | head -1)"
  done
done
