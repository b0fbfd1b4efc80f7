#!/bin/bash
# round-2 GPU session AH: camera and scatter draws in one rejection loop (RT_MERGED_DRAWS) vs
# separate steps, on C2 (pool and items), Cornell and the final scene; then the GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:gpu_tests:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "600:ab_md_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_md0.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
  "600:ab_md_c2i:RT_SCHEDULE=2 python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_md0.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 2" \
  "600:ab_md_c3:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_md0.so --scene 5 --width 800 --height 800 --spp 200 --rounds 2" \
  "600:ab_md_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_md0.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
