#!/bin/bash
# Round-5 GPU sessions (run through gpurun from the repo root; scripts/gpu_session.sh presets).
#   prof   the final build's GPU tests, smoke and PMC passes of C1-C5 (r05f_*); afterwards, here:
#          scripts/sessions_r05.sh pmc  (writes profiles/pmc.json entries + r05_final_c*_pmc.md)
#   lines  the bench lines of C1-C5 (>= 3 timed steps each), the default line and the f32 lines,
#          which read those PMC entries (r05b_*)
# The session letters of the current final build (a4580192: r05f / r05b; 69a9c531: r05aj / r05ak):
# PROF=r05aj_ LINES=r05ak_ by default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROF="${PROF:-r05aj_}"
LINES="${LINES:-r05ak_}"
case "${1:-}" in
prof)
    PREFIX=$PROF scripts/gpu_session.sh tests smoke prof_c1 prof_c2 prof_c3 prof_c4 prof_c5
    ;;
pmc)
    N="round-5 final build (${PROF%_})"
    python scripts/pmc_r02.py bench ${PROF}prof_c1 r05_final_c1 0,1200,800,10,8,1,1 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c2 r05_final_c2 0,1200,800,500,50,1,1 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c3 r05_final_c3 5,800,800,1000,50,1,2 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c4 r05_final_c4 7,1920,1080,1000,50,1,1 "$N" && \
    python scripts/pmc_r02.py bench ${PROF}prof_c5 r05_final_c5 0,4096,4096,4096,50,1,1 "$N"
    ;;
lines)
    PREFIX=$LINES scripts/gpu_session.sh bench bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4
    ;;
*) echo "usage: $0 prof|pmc|lines" >&2; exit 2 ;;
esac
