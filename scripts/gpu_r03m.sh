#!/bin/bash
# round-3 session M: C4 A/B of the shared deferred-walk stack (13 entries instead of 25: 4 blocks per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_session.sh \
  "600:r03m_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
  "400:r03m_tests:python -u -m pytest tests/test_gpu_nesting.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread"
