#!/bin/bash
# world-1 sharded LR: standalone (twice), then the default line's lr legs (lr, s2v, lr.sharded_world1)
# without the headline, to see whether the s2v leg before it changes the sharded step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in ${STANDALONE:-1 2}; do
  timeout -k 10 300 python bench.py --app lr --sharded --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrsh_$i.log 2>&1 || { tail -20 gpurun_out/lrsh_$i.log; exit 1; }
  grep '^{' gpurun_out/lrsh_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('standalone $i', '%.4g' % d['value'], '%.4f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['kernel_ms'].items()})"
done
# the default line (no CPU baselines) in both orders: sharded base before / after the s2v leg
for o in lr_first s2v_first; do
  BENCH_ORDER=$o timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/lrsh_$o.log 2>&1 || { tail -20 gpurun_out/lrsh_$o.log; exit 1; }
  grep '^{' gpurun_out/lrsh_$o.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); q=d['lr']['sharded_world1']; print('$o', 'lr %.4f' % d['lr']['ms_per_step'], 'sharded %.4f' % q['ms_per_step'], q['kernel_ms'], 's2v %.4g' % d['s2v']['value'])"
done
