#!/bin/bash
# round-3 session E: C4 A/B of the deferred instance walk and of the final variant's 16-bit stack (4 waves) after the LDS-layout
# fix, vs the 32-bit stack (LDS-bound 3 waves) and 3-wave registers; C2/C3 of the default build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh \
  "500:r03e_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s32.so $L/librtiow_exp_nodefer.so --scene 7 --width 1920 --height 1080 --spp 100" \
  "200:r03e_phases:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
  "600:r03e_calib:scripts/calib_r02.sh r03e_calib" \
  bench_c2 bench_c3 tests
