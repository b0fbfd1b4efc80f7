#!/bin/bash
# round-2 GPU session AD: traversal loop forms re-measured on HEAD (while-while vs speculative
# while-while vs if-if) on C2 and the final scene
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:ab_loop_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_loop2.so $L/librtiow_exp_loop0.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
  "600:ab_loop_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_loop2.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
