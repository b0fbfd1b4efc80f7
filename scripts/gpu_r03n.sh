#!/bin/bash
# round-3 session N: C4 / C3 / Cornell-smoke A/B: 3-wave build (before the shared stack), the
# shared stack + normal-derived sphere uv without the stack-address rematerialization, and HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh \
  "600:r03n_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_noremat.so $L/librtiow_amd.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
  "400:r03n_ab_c3:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_noremat.so $L/librtiow_amd.so --scene 5 --width 800 --height 800 --spp 200 --rounds 2" \
  "400:r03n_ab_c6:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_noremat.so $L/librtiow_amd.so --scene 6 --width 600 --height 600 --spp 200 --rounds 2" \
  "600:r03n_tests:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
