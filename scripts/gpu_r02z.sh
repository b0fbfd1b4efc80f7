#!/bin/bash
# round-2 GPU session Z: packed-f32 plane products in the LDS node visit (RT_PK_SLAB) A/B on
# C2 and Cornell smoke (the variants it changes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:ab_pk_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_pk.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 4" \
  "600:ab_pk_smoke:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_pk.so --scene 6 --width 600 --height 600 --spp 200 --rounds 3"
