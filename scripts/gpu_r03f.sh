#!/bin/bash
# round-3 session F: C4 stack width x register budget (16/32-bit stack entries, 128/168 VGPRs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh \
  "600:r03f_ab_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_s32.so $L/librtiow_exp_s16w3.so $L/librtiow_exp_s32w3.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 3"
