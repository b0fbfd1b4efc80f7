#!/bin/bash
# round-2 GPU session AM: a sphere-bounded medium's two boundary queries from one quadratic
# (RT_MEDIUM_SPHERE2) vs two sphere tests, on the final scene (and C2 unchanged); then the GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:gpu_tests:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "600:ab_ms_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_ms0.so --scene 7 --width 960 --height 540 --spp 200 --rounds 3" \
  "600:ab_ms_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_ms0.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 2"
