#!/bin/bash
# round-3 session G: GPU tests; C4 A/B of the BLAS top levels staged in LDS; C4 phase timers
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh tests \
  "500:r03g_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_nostage.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 3" \
  "200:r03g_phases:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
