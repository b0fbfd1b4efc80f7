#!/bin/bash
# round-2 GPU session P: per-sample pool block size (tail at small shards), tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "400:shard:python scripts/shard_coherence.py --spp 500 --reps 3 --block-samples 4 8 32"
