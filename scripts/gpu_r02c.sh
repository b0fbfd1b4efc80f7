#!/bin/bash
# round-2 GPU session C: why the item pool issues more instructions than the per-sample pool
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
CNT="--no-cpu-baseline --steps 1 --warmup 0 --count-spp 500"
scripts/gpu_steps.sh \
  "240:c2_items_ch1:RT_SCHEDULE=2 python bench.py --steps 5 --warmup 1 --spp-chunk 1 $NB" \
  "240:c2_items_ch4:RT_SCHEDULE=2 python bench.py --steps 5 --warmup 1 --spp-chunk 4 $NB" \
  "240:c2_items_ch16:RT_SCHEDULE=2 python bench.py --steps 5 --warmup 1 $NB" \
  "240:c2_pool_ch16:RT_SCHEDULE=1 python bench.py --steps 5 --warmup 1 $NB" \
  "240:cnt_items:RT_SCHEDULE=2 python bench.py $CNT" \
  "240:cnt_pool:RT_SCHEDULE=1 python bench.py $CNT" \
  "300:calib:scripts/calib_r02.sh calib3" \
  "600:prof_c2_pool:RT_SCHEDULE=1 PROF_DIR=prof_c2_pool scripts/profile_r02.sh"
