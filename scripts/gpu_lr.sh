cd "${GRAFT_REPO_ROOT}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
mkdir -p gpurun_out
step pytest_lr 600 python -m pytest tests/test_lr_gpu.py tests/test_compat.py -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread || exit $?
step dist2_lr 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 tests/dist_lr_check.py --backend gloo || exit $?
step bench_lr 600 python bench.py --app lr --steps 20 --warmup 3 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step prof_lr 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lr -o run -- python3 bench.py --app lr --steps 20 --warmup 3 || exit $?
