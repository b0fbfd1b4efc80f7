#!/bin/bash
# round-2 GPU session AQ: the final HEAD as the driver runs it — GPU tests, smoke, bench.py with
# no arguments (its roofline quotes this build's PMC entry r02ap_c2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "600:bench_default:python bench.py"
