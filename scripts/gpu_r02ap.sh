#!/bin/bash
# round-2 GPU session AP: 16-bit LDS stack + 5 waves per SIMD in the spheres variant (the new
# default) — GPU tests (incl. both stack widths against the oracle), smoke, benches C2, C1, C5, C4,
# the C2 PMC profile of this build, then bench.py with no arguments
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300:bench_c2:python bench.py --steps 10 --warmup 2" \
  "300:bench_c1:python bench.py --config C1 --steps 20 --warmup 3" \
  "300:bench_c5:python bench.py --config C5 --steps 1 --warmup 0" \
  "300:bench_c4:python bench.py --config C4 --steps 2 --warmup 1 --no-count" \
  "600:prof_c2:PROF_DIR=prof_c2 scripts/profile_r02.sh" \
  "600:bench_default:python bench.py"
