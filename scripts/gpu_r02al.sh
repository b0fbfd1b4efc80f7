#!/bin/bash
# round-2 GPU session AL: sphere radius^2 from the upload (RT_R2) A/B; SAH cost / leaf-size sweep
# at HEAD (after the cheaper LDS node visits), C2 and the final scene, one process each
# (scripts/ab_variants.py --bvh CI:MAXLEAF); then the GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "600:gpu_tests:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "600:ab_r2_c2:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_r20.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 4" \
  "600:ab_r2_c4:python scripts/ab_builds.py $L/librtiow_amd.so $L/librtiow_exp_r20.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2" \
  "600:bvh_c2:python scripts/ab_variants.py --scene 0 --width 1200 --height 800 --spp 100 --rounds 2 --variants 1:1:1 --bvh 1:8,2:8,4:8,1:4,0.5:8,0.5:16" \
  "600:bvh_c4:python scripts/ab_variants.py --scene 7 --width 960 --height 540 --spp 100 --rounds 2 --variants 1:1:1 --bvh 1:8,2:8,1:4,0.5:8"
