#!/bin/bash
# round-2 GPU session AL: SAH cost / leaf-size sweep at HEAD (after the cheaper LDS node visits),
# C2 and the final scene, one process each (scripts/ab_variants.py --bvh CI:MAXLEAF)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "600:bvh_c2:python scripts/ab_variants.py --scene 0 --width 1200 --height 800 --spp 100 --rounds 2 --variants 1:1:1 --bvh 1:8,2:8,4:8,1:4,0.5:8,0.5:16" \
  "600:bvh_c4:python scripts/ab_variants.py --scene 7 --width 960 --height 540 --spp 100 --rounds 2 --variants 1:1:1 --bvh 1:8,2:8,1:4,0.5:8"
