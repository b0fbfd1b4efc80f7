#!/bin/bash
# round-2 GPU session B: schedule A/B on one box, extended VALU calibration, PMC profile of C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "240:ab_c2_items:RT_SCHEDULE=2 python bench.py --steps 10 --warmup 2 $NB" \
  "240:ab_c2_pool:RT_SCHEDULE=1 python bench.py --steps 10 --warmup 2 $NB" \
  "240:ab_c4_items:RT_SCHEDULE=2 python bench.py --config C4 --steps 3 --warmup 1 $NB" \
  "240:ab_c4_pool:RT_SCHEDULE=1 python bench.py --config C4 --steps 3 --warmup 1 $NB" \
  "240:ab_c3_items:RT_SCHEDULE=2 python bench.py --config C3 --steps 5 --warmup 1 $NB" \
  "240:ab_c3_pool:RT_SCHEDULE=1 python bench.py --config C3 --steps 5 --warmup 1 $NB" \
  "300:calib:scripts/calib_r02.sh calib2" \
  "600:prof_c2:PROF_DIR=prof_c2 scripts/profile_r02.sh"
