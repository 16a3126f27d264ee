for d in 0 1 2 3; do SWPS_LR_DIAG=$d timeout -k 10 120 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrdiag_$d.json 2>/dev/null || exit 1; done
