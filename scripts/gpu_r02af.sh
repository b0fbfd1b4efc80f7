#!/bin/bash
# round-2 GPU session AF: sample buffer sized from free HBM (C4 one batch instead of two),
# C5 per-sample pool in ~16 batches vs the item pool; then the GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "300:c4_cap_auto:python bench.py --config C4 --steps 2 --warmup 1 $NB" \
  "300:c4_cap_32g:RT_SAMPLE_BUF_MB=32768 python bench.py --config C4 --steps 2 --warmup 1 $NB" \
  "300:c5_items:python bench.py --config C5 --steps 1 --warmup 0 $NB" \
  "300:c5_pool:RT_SCHEDULE=1 python bench.py --config C5 --steps 1 --warmup 0 $NB" \
  "600:gpu_tests:python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread"
