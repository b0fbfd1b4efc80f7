#!/bin/bash
# round-2 GPU session N: smoke, shard coherence (rank 0 of N on one GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300:shard:python scripts/shard_coherence.py --spp 500 --reps 3"
