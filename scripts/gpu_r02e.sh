#!/bin/bash
# round-2 GPU session E: final-scene feature variant (spills), AUTO schedule; tests, C2/C3/C4 benches, C4 profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:bench_c2:python bench.py --steps 10 --warmup 2 $NB" \
  "300:bench_c3:python bench.py --config C3 --steps 5 --warmup 1 $NB" \
  "300:bench_c4:python bench.py --config C4 --steps 3 --warmup 1 $NB" \
  "300:bench_c4_pool:RT_SCHEDULE=1 python bench.py --config C4 --steps 3 --warmup 1 $NB" \
  "300:bench_c3_items:RT_SCHEDULE=2 python bench.py --config C3 --steps 5 --warmup 1 $NB" \
  "900:prof_c4:PROF_DIR=prof_c4 BENCH_ARGS='--config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-count' scripts/profile_r02.sh"
