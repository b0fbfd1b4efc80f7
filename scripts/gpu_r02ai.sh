#!/bin/bash
# round-2 GPU session AI: Dielectric 1/ir and Schlick r0 from the upload (RT_DIEL_CONST) vs per hit,
# on C2 and the final scene; then the GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:gpu_tests:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "600:ab_dc_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_dc0.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
  "600:ab_dc_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_dc0.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
