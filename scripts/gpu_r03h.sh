#!/bin/bash
# round-3 session H: C4 A/B of how many BLAS nodes to stage in LDS (256 = the LDS budget, 64, 16, none)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh \
  "600:r03h_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_b64.so $L/librtiow_exp_b16.so $L/librtiow_exp_nostage.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2"
