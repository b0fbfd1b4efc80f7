#!/bin/bash
# round-2 GPU session F: item-pool block groups (coherence) A/B on C2, tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "240:c2_items_g1:RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 $NB" \
  "240:c2_items_g2:RT_ITEM_GROUP=2 RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 $NB" \
  "240:c2_items_g4:RT_ITEM_GROUP=4 RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 $NB" \
  "240:c2_items_g8ch4:RT_ITEM_GROUP=8 RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 --spp-chunk 4 $NB" \
  "240:c2_items_g1ch4:RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 --spp-chunk 4 $NB" \
  "240:c2_auto:python bench.py --steps 6 --warmup 1 $NB" \
  "240:c2_items_cnt:RT_SCHEDULE=2 python bench.py --steps 1 --warmup 0 --no-cpu-baseline" \
  "240:c2_items_g4_cnt:RT_ITEM_GROUP=4 RT_SCHEDULE=2 python bench.py --steps 1 --warmup 0 --no-cpu-baseline" \
  "240:c2_pool_cnt:RT_SCHEDULE=1 python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
