#!/bin/bash
# round-2 GPU session Y: RT_DONE sentinel at the bottom of each walk (pops without an empty test): tests, A/B vs HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "600:ab_c2:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 4" \
  "600:ab_c3:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 5 --width 800 --height 800 --spp 200 --rounds 3" \
  "600:ab_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
