#!/bin/bash
# round-3 session I: the committed build end to end — GPU tests, smoke, C1-C5 f64 and C2-C4 f32
# bench lines, count-variant phase shares (C2, C4 f64, C4 f32)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PREFIX=r03i_ scripts/gpu_session.sh tests smoke bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 f32_c2 f32_c3 f32_c4 \
  "200:r03i_phases_c2:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
  "300:r03i_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8" \
  "300:r03i_phases_c4_f32:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8 --precision f32"
