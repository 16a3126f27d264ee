set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lr_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/lr_tests.log 2>&1; rc=$?
tail -5 gpurun_out/lr_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for t in 0 1; do SWPS_LR_TILES=$t timeout -k 10 120 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrt_${t}_$r.json 2>/dev/null || exit 1; done
done
bash scripts/lr_prof_quick.sh
