#!/bin/bash
# round-2 GPU session AJ2: far-plane min as v_med3(fz, t_max, -inf from an SGPR) (RT_MED3) vs
# fminf, and on top of it the pre-scaled stack pointer (RT_SPTR), on C2 and the final scene;
# then the GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:gpu_tests:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "600:ab_med_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_med0.so $L/librtiow_exp_sp1.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 4" \
  "600:ab_med_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_med0.so $L/librtiow_exp_sp1.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
