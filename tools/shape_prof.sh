cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for n in 32 64 128 256; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shp$n -o run -- python tools/shape_probe.py --only "lognormal, $n trees" --steps 50 > gpurun_out/shp$n.log 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shp128 -o run -- python tools/shape_probe.py --only "mean 256" --steps 50 > gpurun_out/shp128.log 2>&1
