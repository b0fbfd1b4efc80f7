#!/bin/bash
# round-2 GPU session AK: the measured HEAD — GPU tests, smoke, benches C1-C5 (f64) and C2-C4
# (f32), PMC profiles of C2, C3 and C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300:bench_c2:python bench.py --steps 10 --warmup 2" \
  "300:bench_c1:python bench.py --config C1 --steps 20 --warmup 3" \
  "300:bench_c3:python bench.py --config C3 --steps 5 --warmup 1" \
  "300:bench_c4:python bench.py --config C4 --steps 2 --warmup 1" \
  "300:bench_c5:python bench.py --config C5 --steps 1 --warmup 0" \
  "300:f32_c2:python bench.py --steps 10 --warmup 2 --precision f32 $NB" \
  "300:f32_c3:python bench.py --config C3 --steps 5 --warmup 1 --precision f32 $NB" \
  "300:f32_c4:python bench.py --config C4 --steps 2 --warmup 1 --precision f32 $NB" \
  "600:prof_c2:PROF_DIR=prof_c2 scripts/profile_r02.sh" \
  "600:prof_c3:PROF_DIR=prof_c3 BENCH_ARGS='--config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-count' scripts/profile_r02.sh" \
  "900:prof_c4:PROF_DIR=prof_c4 BENCH_ARGS='--config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-count' scripts/profile_r02.sh"
