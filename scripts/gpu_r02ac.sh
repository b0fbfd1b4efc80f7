#!/bin/bash
# round-2 GPU session AC: pre_leaf in the spheres variants only: tests, A/B on C2 and C5-like items
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "600:ab_hoist_c2:python scripts/ab_builds.py $L/librtiow_exp_nohoist.so $L/librtiow_amd.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 4" \
  "600:ab_hoist_c2i:RT_SCHEDULE=2 python scripts/ab_builds.py $L/librtiow_exp_nohoist.so $L/librtiow_amd.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3"
