#!/bin/bash
# round-2 GPU session AB: huge root-child leaf tested before the TLAS walk (SceneDev.pre_leaf):
# tests, A/B vs the same build without it on C2 and the final scene
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "600:ab_hoist_c2:python scripts/ab_builds.py $L/librtiow_exp_nohoist.so $L/librtiow_amd.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 4" \
  "600:ab_hoist_c4:python scripts/ab_builds.py $L/librtiow_exp_nohoist.so $L/librtiow_amd.so --scene 7 --width 960 --height 540 --spp 200 --rounds 3"
