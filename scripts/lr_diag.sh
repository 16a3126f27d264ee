# SWPS_LR_DIAG timing experiments (wrong results): 1 forward without weight
# gathers, 2 without the ordered chain, 4 k_lr_records without its e gathers (SWPS_LR_TILES=0),
# 8 k_lr_tiles without its piece ends, 16 without the e slice fill
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in ${DIAGS:-0 1 2 8 16 24}; do SWPS_LR_DIAG=$d timeout -k 10 120 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrdiag_$d.json 2>/dev/null || exit 1; done
