#!/bin/bash
# round-3 session S: the committed build end to end — GPU tests, smoke, bench lines C1-C5 (f64) and
# C2-C4 (f32), PMC profiles of C2 / C3 / C4 (the roofline bench.py quotes for this source hash),
# C4 phase shares
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PREFIX=r03s_ scripts/gpu_session.sh tests smoke bench bench_c4 prof_c2 prof_c4 bench_c1 bench_c3 bench_c5 prof_c3 f32_c2 f32_c3 f32_c4 \
  "300:r03s_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
