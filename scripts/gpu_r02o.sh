#!/bin/bash
# round-2 GPU session O: row-band shards (tests, coherence per GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:shard:python scripts/shard_coherence.py --spp 500 --reps 3"
