cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for rep in 1 2; do for v in 512 1024 256; do
SWPS_LR_NHOT=$v timeout -k 10 200 python bench.py --app lr --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/lrab_$v.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('gpurun_out/lrab_$v.json').read().strip().splitlines()[-1]); print('NHOT=$v', d['value'], d['ms_per_step'], json.dumps(d['kernel_ms']))"
done; done
