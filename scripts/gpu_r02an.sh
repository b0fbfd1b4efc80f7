#!/bin/bash
# round-2 GPU session AN: the final HEAD as the driver runs it — GPU tests, smoke, and
# bench.py with no arguments (its roofline must quote this build's PMC entry)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_steps.sh \
  "900:gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "600:bench_default:python bench.py"
