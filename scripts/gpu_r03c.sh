#!/bin/bash
# round-3 session C: phase timers (count variant) of C2, C4, C3; the counters rocprofv3 offers on
# this box; a PC-sampling trial on a C4-shaped render (last: a failure there stops nothing else)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
scripts/gpu_session.sh \
  "300:r03c_phases:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16 && python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8 && python scripts/phases.py --scene 5 --width 800 --height 800 --spp 16" \
  "120:r03c_counters:rocprofv3 -L" \
  "180:r03c_pcs:rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --output-format csv -d gpurun_out/r03c_pcs -o pcs -- python3 bench.py --config C4 --width 960 --height 540 --spp 50 --steps 1 --warmup 0 --no-cpu-baseline --no-count"
