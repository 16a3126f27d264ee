cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lrq -o run -- python3 bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrq.log 2>&1 || exit $?
cp gpurun_out/lrq/run_kernel_stats.csv gpurun_out/lrq_stats.csv
rm -rf gpurun_out/lrq
