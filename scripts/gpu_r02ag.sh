#!/bin/bash
# round-2 GPU session AG: finish_ray once per bounce iteration (RT_FINISH_AT_TRACE) vs in the
# camera and shading steps, on C2, Cornell and the final scene; then the GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:ab_fin_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_fin0.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
  "600:ab_fin_c3:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_fin0.so --scene 5 --width 800 --height 800 --spp 200 --rounds 2" \
  "600:ab_fin_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_fin0.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2" \
  "600:gpu_tests:python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread"
