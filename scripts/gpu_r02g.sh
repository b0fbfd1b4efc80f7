#!/bin/bash
# round-2 GPU session G: f32 mode tests + bench; block grouping A/B (pool and items) on C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "240:c2_f32:python bench.py --steps 6 --warmup 1 --precision f32 $NB" \
  "240:c2_pool_b2:RT_BLOCK_CHUNKS=2 RT_SCHEDULE=1 python bench.py --steps 6 --warmup 1 $NB" \
  "240:c2_pool_b4:RT_BLOCK_CHUNKS=4 RT_SCHEDULE=1 python bench.py --steps 6 --warmup 1 $NB" \
  "240:c2_pool_ch8b4:RT_BLOCK_CHUNKS=4 RT_SCHEDULE=1 python bench.py --steps 6 --warmup 1 --spp-chunk 8 $NB" \
  "240:c2_items_ch4b16:RT_BLOCK_CHUNKS=16 RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 --spp-chunk 4 $NB" \
  "240:c2_items_ch2b16:RT_BLOCK_CHUNKS=16 RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 --spp-chunk 2 $NB" \
  "240:c2_items_ch8b4:RT_BLOCK_CHUNKS=4 RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 --spp-chunk 8 $NB" \
  "240:c2_items_ch4b4:RT_BLOCK_CHUNKS=4 RT_SCHEDULE=2 python bench.py --steps 6 --warmup 1 --spp-chunk 4 $NB" \
  "300:c4_f32:python bench.py --config C4 --steps 2 --warmup 1 --precision f32 $NB" \
  "300:c3_f32:python bench.py --config C3 --steps 3 --warmup 1 --precision f32 $NB"
