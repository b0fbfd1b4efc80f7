#!/bin/bash
# round-2 GPU session D (re-entry): GPU tests on HEAD, headline bench, schedule A/B, PMC profile of HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "240:warm:python -c 'import torch; print(torch.__version__, torch.cuda.device_count())'" \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:bench_c2:python bench.py --steps 10 --warmup 2" \
  "240:ab_c2_pool:RT_SCHEDULE=1 python bench.py --steps 10 --warmup 2 $NB" \
  "240:ab_c2_chunks:RT_SCHEDULE=0 python bench.py --steps 10 --warmup 2 $NB" \
  "600:prof_c2:PROF_DIR=prof_c2 scripts/profile_r02.sh"
