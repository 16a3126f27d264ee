# A/B of the fixed-point step's bucket width: build libswps_vb<N>.so copies with kLrFxVB = N first (swps_lr.hip), then run this on one box
cd "${GRAFT_REPO_ROOT}"
L=swiftmpi_amd/lib
for rep in 1 2; do for v in ${VB_LIST:-12 11}; do
cp $L/libswps_vb$v.so $L/libswps.so
timeout -k 10 200 python bench.py --app lr --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/vb_$v.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('gpurun_out/vb_$v.json').read().strip().splitlines()[-1]); print('VB=$v', d['value'], d['ms_per_step'], json.dumps(d['kernel_ms']))"
done; done
cp $L/libswps_vb12.so $L/libswps.so
