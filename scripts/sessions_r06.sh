#!/bin/bash
# Round-6 GPU sessions (run through gpurun from the repo root; scripts/gpu_session.sh presets).
#   prof1  the final build's GPU tests, smoke and the PMC passes of C1-C3
#   prof2  the PMC passes of C4 and C5 (a call is at most 20 minutes)
#   pmc    (here, afterwards) profiles/pmc.json entries + r06_final_c*_pmc.md from them
#   lines  the bench lines of C1-C5 (>= 3 timed steps each), the default line and the f32 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROF="${PROF:-r06p_}"
LINES="${LINES:-r06q_}"
case "${1:-}" in
prof1) PREFIX=$PROF scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 ;;
prof2) PREFIX=$PROF scripts/gpu_session.sh prof_c4 prof_c5 ;;
pmc)
    N="round-6 final build (${PROF%_})"
    python scripts/pmc_r02.py bench ${PROF}prof_c1 r06_final_c1 0,1200,800,10,8,1,1 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c2 r06_final_c2 0,1200,800,500,50,1,1 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c3 r06_final_c3 5,800,800,1000,50,1,2 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c4 r06_final_c4 7,1920,1080,1000,50,1,1 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c5 r06_final_c5 0,4096,4096,4096,50,1,1 "$N"
    ;;
lines) PREFIX=$LINES scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4 ;;
*) echo "usage: $0 prof1|prof2|pmc|lines" >&2; exit 2 ;;
esac
