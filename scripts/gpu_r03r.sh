#!/bin/bash
# round-3 session R: final-scene variant in 512-thread workgroups (one LDS copy of the TLAS per
# 8 waves: RT_BLOCK_FINAL=512), with the BLAS staging cap at 64 nodes and lifted; GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh \
  "600:r03r_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_b512.so $L/librtiow_exp_b512all.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
  tests
