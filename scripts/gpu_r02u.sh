#!/bin/bash
# round-2 GPU session U: per-box reciprocals in box_t (RT_BOX_RCP) A/B on C3, smoke, final; tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "600:ab_boxrcp_c3:python scripts/ab_builds.py $L/librtiow_exp_nobox.so $L/librtiow_amd.so --scene 5 --width 800 --height 800 --spp 200 --rounds 3" \
  "600:ab_boxrcp_smoke:python scripts/ab_builds.py $L/librtiow_exp_nobox.so $L/librtiow_amd.so --scene 6 --width 600 --height 600 --spp 200 --rounds 2" \
  "600:ab_boxrcp_c4:python scripts/ab_builds.py $L/librtiow_exp_nobox.so $L/librtiow_amd.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
