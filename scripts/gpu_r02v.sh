#!/bin/bash
# round-2 GPU session V (re-entry): GPU tests and the C2 bench on HEAD (per-box reciprocals)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:bench_c2:python bench.py --steps 10 --warmup 2"
