#!/bin/bash
# round 6 evidence: rocprof kernel summaries + PMC passes + bench lines of the legs round 6 changed
# (LR, sent2vec) and the ones the verdict asked to refresh (config 4), the headline and B = 100;
# then the B = 100 kernel timeline (gaps between dependent launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r06 LEGS="${LEGS:-lr w2v_bfp32 w2v_config4 s2v w2v_b100}" bash scripts/gpu_profile.sh || exit $?
bash scripts/r6_probe_b100.sh
