#!/bin/bash
# round-3 session L: VALU calibration with the kernel-mix replays (KMIX_C2 / KMIX_C4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh "600:r03l_calib:scripts/calib_r02.sh r03l_calib"
