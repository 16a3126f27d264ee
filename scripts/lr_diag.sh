# SWPS_LR_DIAG timing experiments: 1 forward without weight gathers, 2 without
# the ordered chain, 4 k_lr_records without its e gathers (coalesced reads instead)
for d in ${DIAGS:-0 1 2 4 5}; do SWPS_LR_DIAG=$d timeout -k 10 120 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrdiag_$d.json 2>/dev/null || exit 1; done
