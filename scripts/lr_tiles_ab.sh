# LR row tiles: GPU tests, then same-box A/B of the record path and the tile block sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lr_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/lr_tests.log 2>&1; rc=$?
tail -5 gpurun_out/lr_tests.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-SWPS_LR_TILES=0;SWPS_LR_TILE_CHUNK=1024;SWPS_LR_TILE_CHUNK=2048;SWPS_LR_TILE_CHUNK=4096}" REPS=2 bash scripts/lr_ab.sh
