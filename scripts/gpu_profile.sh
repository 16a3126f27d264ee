#!/bin/bash
# rocprofv3 evidence for the bench lines, per leg, written to
# gpurun_out/profiles_$TAG/ (copy into profiles/ afterwards):
#   <tag>_<leg>_kernel_stats.csv   kernel-trace + stats of the leg's command
#   <tag>_bench_<leg>_traced.json  the bench JSON line of that traced process
#   <tag>_pmc_<leg>.json           separate --pmc passes of the same command
#                                  (read requests by size; WRITE_SIZE; for the
#                                  headline also FETCH_SIZE as a cross-check),
#                                  summarised by scripts/pmc_summary.py
#   <tag>_bench_<leg>.json         the same command without the profiler, its
#                                  roofline.traffic read from that summary
# LEGS selects legs (default: all).  Each step runs under its own time limit;
# the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
OUT=gpurun_out/profiles_$TAG
mkdir -p gpurun_out "$OUT" profiles
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
LEGS=${LEGS:-"w2v_bfp32 w2v_bfp40 w2v_b100 w2v_parity w2v_fast lr s2v w2v_config4 w2v_sharded"}
READS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
W2V="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0 --no-app-legs"
W2VCFG='"app": "w2v", "dim": 300, "dtype": "f32", "world": 1, "line_len": 1000, "sampler": "table"'
TEXT8='"tokens": 17005207, "vocab": 253854'
leg() {  # name last(N|launches) config-json args...
  local name=$1 last=$2 cfg=$3; shift 3
  run prof_$name 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- python3 "$@" || exit $?
  cp gpurun_out/prof_$name/run_kernel_stats.csv "$OUT/${TAG}_${name}_kernel_stats.csv"
  grep '^{' gpurun_out/prof_$name.log | tail -1 > "$OUT/${TAG}_bench_${name}_traced.json"
  if [ "$last" = launches ]; then
    last=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['launches'])" "$OUT/${TAG}_bench_${name}_traced.json") || exit 1
  fi
  local dirs="gpurun_out/pmc_rd_$name gpurun_out/pmc_wr_$name"
  run pmc_rd_$name 900 rocprofv3 --pmc $READS --kernel-trace --output-format csv -d gpurun_out/pmc_rd_$name -o run -- python3 "$@" || exit $?
  run pmc_wr_$name 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_wr_$name -o run -- python3 "$@" || exit $?
  if [ -n "$FETCH" ]; then
    run pmc_fe_$name 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fe_$name -o run -- python3 "$@" || exit $?
    dirs="$dirs gpurun_out/pmc_fe_$name"
  fi
  python3 scripts/pmc_summary.py "$OUT/${TAG}_pmc_${name}.json" $dirs --last "$last" --cmd "python3 $*" --config "$cfg" || exit $?
  cp "$OUT/${TAG}_pmc_${name}.json" profiles/
  run bench_$name 900 python3 "$@" || exit $?
  grep '^{' gpurun_out/bench_$name.log | tail -1 > "$OUT/${TAG}_bench_${name}.json"
  # the per-dispatch traces are tens of MB each: only the summaries travel back
  rm -rf gpurun_out/prof_$name gpurun_out/pmc_rd_$name gpurun_out/pmc_wr_$name gpurun_out/pmc_fe_$name
}
for L in $LEGS; do
  case $L in
    w2v_bfp32) FETCH=1 leg $L 20 "{$W2VCFG, $TEXT8, \"minibatch\": 5000, \"mode\": \"bfp32\", \"sharded\": false}" $W2V ;;
    w2v_bfp40) leg $L 20 "{$W2VCFG, $TEXT8, \"minibatch\": 5000, \"mode\": \"bfp40\", \"sharded\": false}" $W2V --precision bfp40 ;;
    w2v_b100) leg $L 200 "{$W2VCFG, $TEXT8, \"minibatch\": 100, \"mode\": \"bfp32\", \"sharded\": false}" \
                bench.py --gpus 1 --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline --no-parity-leg --config1-steps 0 --no-app-legs ;;
    w2v_parity) leg $L 20 "{$W2VCFG, $TEXT8, \"minibatch\": 5000, \"mode\": \"parity\", \"sharded\": false}" $W2V --parity ;;
    w2v_fast) leg $L 20 "{$W2VCFG, $TEXT8, \"minibatch\": 5000, \"mode\": \"fast\", \"sharded\": false}" $W2V --precision fast ;;
    lr) leg $L 20 '{"app": "lr", "lr_batch": 65536, "exact": false, "world": 1, "sharded": false, "plan": "none"}' \
          bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline ;;
    # 124 + 31 minibatches of 8193 docs: every docs launch (one per 31 minibatches: 262,144 docs at
    # most) the same size, so rocprof's per-launch average and the profiled pass's agree
    s2v) leg $L launches '{"app": "s2v", "s2v_docs": 8192, "dim": 300, "world": 1}' \
           bench.py --app s2v --steps 124 --warmup 31 --no-cpu-baseline ;;
    w2v_config4) leg $L 20 "{$W2VCFG, \"tokens\": 125000000, \"vocab\": 1000000, \"minibatch\": 5000, \"mode\": \"bfp32\", \"sharded\": false}" \
                   $W2V --tokens 125000000 --vocab 1000000 ;;
    w2v_sharded) leg $L 20 "{$W2VCFG, $TEXT8, \"minibatch\": 5000, \"mode\": \"bfp32\", \"sharded\": true}" $W2V --sharded ;;
    *) echo "unknown leg $L"; exit 2 ;;
  esac
done
ls -la "$OUT"
