#!/bin/bash
# round-2 GPU session K: packed-f32 slab A/B (spheres variant, C2), rect reciprocals A/B (C3), GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "600:ab_pk:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_pk.so --rounds 3" \
  "600:ab_rcp:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_norcp.so --scene 5 --width 800 --height 800 --spp 200 --rounds 3"
