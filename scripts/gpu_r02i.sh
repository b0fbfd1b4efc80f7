#!/bin/bash
# round-2 GPU session I: f32 origin offset; f32 tests; C4/C2/C3 f32 perf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "600:gpu_tests_f32:python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_parity.py -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:c4_f32_960:python bench.py --config C4 --width 960 --height 540 --spp 200 --steps 3 --warmup 1 --precision f32 $NB" \
  "300:c2_f32:python bench.py --steps 6 --warmup 1 --precision f32 $NB" \
  "300:c3_f32:python bench.py --config C3 --steps 3 --warmup 1 --precision f32 $NB"
