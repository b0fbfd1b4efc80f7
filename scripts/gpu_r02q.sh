#!/bin/bash
# round-2 GPU session Q: static spheres as zero-velocity moving spheres (A/B on C2), tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "600:ab_sph:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_new.so --rounds 3" \
  "600:ab_sph_final:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_exp_new.so --scene 7 --width 960 --height 540 --spp 200 --rounds 2"
