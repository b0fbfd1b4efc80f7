#!/bin/bash
# round-3 session J: PMC profiles (kernel trace + SQ/TCC passes) of C2 and C4 at the committed build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PREFIX=r03j_ scripts/gpu_session.sh prof_c2 prof_c4
