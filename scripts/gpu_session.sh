#!/bin/bash
# One GPU session on the box (run through gpurun from the repo root): named steps in order,
# each under its own time limit (scripts/gpu_steps.sh: a fault, abort, segfault or timeout
# stops the session). Replaces round 2's one-off gpu_r02*.sh launchers.
#
# usage: scripts/gpu_session.sh STEP [STEP ...]
#   STEP is a preset name below, or a raw "<seconds>:<name>:<command>" spec.
#   tests            pytest -m gpu (the driver's GPU tier)
#   smoke            __graft_entry__.smoke()
#   bench            bench.py with no arguments (the driver's bench line)
#   bench_c1..c5     bench.py --config Cn (f64)
#   f32_c2..c4       bench.py --config Cn --precision f32
#   prof_c1..c5      scripts/profile_r02.sh on that config (kernel trace + PMC passes)
#   calib            scripts/calib_r02.sh (VALU issue-rate calibration through rocprofv3)
# env: PREFIX (log-name prefix, e.g. r03a_). Round 3 sessions: scripts/sessions_r03.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PREFIX:-}
NB="--no-cpu-baseline --no-count"
specs=()
for s in "$@"; do
    case "$s" in
    tests) specs+=("900:${P}gpu_tests:python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread") ;;
    smoke) specs+=("300:${P}smoke:python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) specs+=("600:${P}bench_default:python bench.py") ;;
    bench_c1) specs+=("300:${P}bench_c1:python bench.py --config C1 --steps 20 --warmup 3") ;;
    bench_c2) specs+=("300:${P}bench_c2:python bench.py --steps 10 --warmup 2") ;;
    bench_c3) specs+=("300:${P}bench_c3:python bench.py --config C3 --steps 5 --warmup 1") ;;
    bench_c4) specs+=("400:${P}bench_c4:python bench.py --config C4 --steps 3 --warmup 1") ;;
    bench_c5) specs+=("600:${P}bench_c5:python bench.py --config C5 --steps 3 --warmup 1") ;;
    f32_c2) specs+=("300:${P}f32_c2:python bench.py --steps 10 --warmup 2 --precision f32 $NB") ;;
    f32_c3) specs+=("300:${P}f32_c3:python bench.py --config C3 --steps 5 --warmup 1 --precision f32 $NB") ;;
    f32_c4) specs+=("300:${P}f32_c4:python bench.py --config C4 --steps 3 --warmup 1 --precision f32 $NB") ;;
    prof_c1) specs+=("500:${P}prof_c1:PROF_DIR=${P}prof_c1 BENCH_ARGS='--config C1 --steps 2 --warmup 1 $NB' scripts/profile_r02.sh") ;;
    prof_c2) specs+=("700:${P}prof_c2:PROF_DIR=${P}prof_c2 scripts/profile_r02.sh") ;;
    prof_c3) specs+=("700:${P}prof_c3:PROF_DIR=${P}prof_c3 BENCH_ARGS='--config C3 --steps 1 --warmup 0 $NB' scripts/profile_r02.sh") ;;
    prof_c4) specs+=("900:${P}prof_c4:PROF_DIR=${P}prof_c4 BENCH_ARGS='--config C4 --steps 1 --warmup 0 $NB' scripts/profile_r02.sh") ;;
    prof_c5) specs+=("900:${P}prof_c5:PROF_DIR=${P}prof_c5 BENCH_ARGS='--config C5 --steps 1 --warmup 0 $NB' scripts/profile_r02.sh") ;;
    calib) specs+=("600:${P}calib:scripts/calib_r02.sh") ;;
    *:*:*) specs+=("$s") ;;
    *) echo "unknown step: $s" >&2; exit 2 ;;
    esac
done
exec scripts/gpu_steps.sh "${specs[@]}"
