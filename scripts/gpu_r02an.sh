#!/bin/bash
# round-2 GPU session AN: the final HEAD — GPU tests, smoke, benches C2 and C4, PMC profiles of
# C2 (the driver's bench workload) and C4 on this build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300:bench_c2:python bench.py --steps 10 --warmup 2" \
  "300:bench_c4:python bench.py --config C4 --steps 2 --warmup 1" \
  "600:prof_c2:PROF_DIR=prof_c2 scripts/profile_r02.sh" \
  "900:prof_c4:PROF_DIR=prof_c4 BENCH_ARGS='--config C4 --steps 1 --warmup 0 --no-cpu-baseline --no-count' scripts/profile_r02.sh"
