#!/bin/bash
# round-2 GPU session T: Cornell variants without the nested BLAS walk, f64 slabs for node-free
# scenes (4 waves per SIMD): tests, A/B against HEAD's build on C3, smoke, final scene
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "600:ab_occ_c3:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 5 --width 800 --height 800 --spp 200 --rounds 3" \
  "600:ab_occ_smoke:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 6 --width 600 --height 600 --spp 200 --rounds 2" \
  "600:ab_occ_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
