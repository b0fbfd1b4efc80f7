#!/bin/bash
# round-3 session D: GPU tests of the relative-BLAS / 16-bit-stack final variant; A/B of the
# final variant's 16-bit stack (4 waves) vs 32-bit (LDS-bound 3 waves) vs 3-wave registers (C4);
# rect / box reciprocal divisions (C3, C4, Cornell smoke); phase timers of C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh tests \
  "500:r03d_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s32.so $L/librtiow_exp_w3.so $L/librtiow_exp_rectrcp.so $L/librtiow_exp_boxrcp.so --scene 7 --width 1920 --height 1080 --spp 100" \
  "300:r03d_ab_c3:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_rectrcp.so $L/librtiow_exp_boxrcp.so --scene 5 --width 800 --height 800 --spp 200" \
  "300:r03d_ab_c6:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_rectrcp.so $L/librtiow_exp_boxrcp.so --scene 6 --width 600 --height 600 --spp 200" \
  "200:r03d_phases:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
