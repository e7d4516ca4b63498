set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k spmm > gpurun_out/spmm_tests.log 2>&1
for v in ${VARIANTS:-wave10 wave7 wave5 block}; do
  echo "== $v" >> gpurun_out/agg_ab.txt
  BGCN_SPMM_WIDE=$v timeout -k 10 120 python tools/agg_probe.py >> gpurun_out/agg_ab.txt 2>&1
done
