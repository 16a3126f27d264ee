#!/bin/bash
# rocprofv3 evidence for the bench line, written to gpurun_out/profiles_$TAG/
# (copy into profiles/ afterwards):
#   * kernel-trace + stats of the headline command (the driver's --steps 20
#     --warmup 5; the extra legs off so the profiled pass's launches are the
#     last ones of each kernel) -> <tag>_w2v_fast_kernel_stats.csv and the
#     bench JSON line of that same traced process -> <tag>_bench_w2v_traced.json
#   * FETCH_SIZE and WRITE_SIZE in separate --pmc passes of the same command
#     (never combined with other tracing) -> <tag>_pmc_w2v_fast.json
#   * the B = 100 minibatch, parity mode and LR (config 3) kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
OUT=gpurun_out/profiles_$TAG
mkdir -p gpurun_out "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
B="$R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0"
run prof_fast 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fast -o run -- python3 $B || exit $?
cp gpurun_out/prof_fast/run_kernel_stats.csv "$OUT/${TAG}_w2v_fast_kernel_stats.csv"
grep '^{' gpurun_out/prof_fast.log | tail -1 > "$OUT/${TAG}_bench_w2v_traced.json"
run pmc_fetch_fast 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_fast -o run -- python3 $B || exit $?
run pmc_write_fast 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_fast -o run -- python3 $B || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_fetch_fast gpurun_out/pmc_write_fast "$OUT/${TAG}_pmc_w2v_fast.json" \
  --last 16 --cmd "python3 bench.py --gpus 1 --steps 20 --warmup 5 (legs off)" \
  --config '{"minibatch": 5000, "dim": 300, "dtype": "f32", "mode": "fast", "world": 1, "tokens": 17005207, "vocab": 253854, "line_len": 1000}' || exit $?
run prof_b100 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b100 -o run -- python3 $R/bench.py --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline --no-parity-leg || exit $?
cp gpurun_out/prof_b100/run_kernel_stats.csv "$OUT/${TAG}_w2v_b100_kernel_stats.csv"
grep '^{' gpurun_out/prof_b100.log | tail -1 > "$OUT/${TAG}_bench_w2v_b100_traced.json"
run prof_parity 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_parity -o run -- python3 $B --parity || exit $?
cp gpurun_out/prof_parity/run_kernel_stats.csv "$OUT/${TAG}_w2v_parity_kernel_stats.csv"
run prof_lr 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lr -o run -- python3 $R/bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline || exit $?
cp gpurun_out/prof_lr/run_kernel_stats.csv "$OUT/${TAG}_lr_kernel_stats.csv"
grep '^{' gpurun_out/prof_lr.log | tail -1 > "$OUT/${TAG}_bench_lr_traced.json"
ls -la "$OUT"
# sent2vec (config-5 per-rank shape) and word2vec at config 4's per-rank shape (V = 1M, 125M tokens)
run bench_s2v 900 python3 $R/bench.py --app s2v --steps 150 --warmup 3 || exit $?  # 8192 x 153 = 1.25M docs: config 5 per rank
grep '^{' gpurun_out/bench_s2v.log | tail -1 > "$OUT/${TAG}_bench_s2v_config5_per_rank.json"
run bench_c4 900 python3 $R/bench.py --tokens 125000000 --vocab 1000000 --steps 20 --warmup 5 --no-parity-leg --b100-steps 0 --no-cpu-baseline || exit $?
grep '^{' gpurun_out/bench_c4.log | tail -1 > "$OUT/${TAG}_bench_w2v_config4_per_rank.json"
run bench_sharded 600 python3 $R/bench.py --sharded --steps 20 --warmup 5 --b100-steps 0 --no-parity-leg --no-cpu-baseline || exit $?
grep '^{' gpurun_out/bench_sharded.log | tail -1 > "$OUT/${TAG}_bench_w2v_sharded_native_world1.json"
run bench_default 900 python3 $R/bench.py --steps 20 --warmup 5 || exit $?
grep '^{' gpurun_out/bench_default.log | tail -1 > "$OUT/${TAG}_bench_w2v_default.json"
ls -la "$OUT"
