#!/bin/bash
# round-2 GPU session A: GPU tests, headline bench, counter list, VALU calibration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "240:warm:python -c 'import torch; print(torch.__version__, torch.cuda.device_count())'" \
  "600:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "240:bench_c2:python bench.py --steps 20 --warmup 5" \
  "60:counters:rocprofv3 -L" \
  "300:calib:scripts/calib_r02.sh calib"
