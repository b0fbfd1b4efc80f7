#!/bin/bash
# round-2 GPU session X: shard coherence on HEAD (row_block 1 / 2 / 4 at N = 1..8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "600:shard:python scripts/shard_coherence.py --spp 500 --reps 3 --row-blocks 1 2 4"
