#!/bin/bash
# round-2 GPU session H: f32 fog-step fix; f32 tests; C4 f32 vs f64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NB="--no-cpu-baseline --no-count"
scripts/gpu_steps.sh \
  "600:gpu_tests_f32:python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_parity.py -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:c4_f32:python bench.py --config C4 --steps 2 --warmup 1 --precision f32 $NB" \
  "300:c4_f64:python bench.py --config C4 --steps 2 --warmup 1 $NB" \
  "300:c4_f32_960:python bench.py --config C4 --width 960 --height 540 --spp 200 --steps 3 --warmup 1 --precision f32 $NB" \
  "300:c4_f64_960:python bench.py --config C4 --width 960 --height 540 --spp 200 --steps 3 --warmup 1 $NB"
