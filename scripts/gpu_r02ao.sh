#!/bin/bash
# round-2 GPU session AO (experiment): 16-bit LDS stack entries in the spheres variant
# (RT_STACK16), at 4 and at 5 waves per SIMD (RT_MIN_WAVES_SPHERES=5), vs HEAD on C2 and C1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:ab_s16_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s16w4.so $L/librtiow_exp_s16w5.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
  "600:ab_s16_c2i:RT_SCHEDULE=2 python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s16w5.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 2"
