#!/bin/bash
# round-3 session P: per-sample buffer in tiled order (tiled_record) vs [sample][pixel]: C2 / C4 A/B,
# the 4-wide TLAS (RT_WIDE) on C2 with its count-variant phases, WRITE_SIZE of C2 and C4 on the new
# build, GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
NB="--no-cpu-baseline --no-count"
W="timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv"
scripts/gpu_session.sh \
  "300:r03p_w4_smoke:RT_LIB_PATH=$PWD/$L/librtiow_exp_w4.so python -c 'import __graft_entry__ as g; g.smoke()'" \
  "400:r03p_ab_c2:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so $L/librtiow_exp_w4.so --scene 0 --width 1200 --height 800 --spp 100 --rounds 3" \
  "200:r03p_phases_c2_w4:RT_LIB_PATH=$PWD/$L/librtiow_exp_w4.so python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
  "200:r03p_phases_c2:python scripts/phases.py --scene 0 --width 1200 --height 800 --spp 16" \
  "600:r03p_ab_c4:python scripts/ab_builds.py $L/librtiow_exp_old.so $L/librtiow_amd.so --scene 7 --width 1920 --height 1080 --spp 100 --rounds 2" \
  "300:r03p_write_c2:export TMPDIR=/tmp; $W -d gpurun_out/r03p_write_c2 -o w -- python3 bench.py --steps 1 --warmup 0 $NB" \
  "300:r03p_write_c4:export TMPDIR=/tmp; $W -d gpurun_out/r03p_write_c4 -o w -- python3 bench.py --config C4 --steps 1 --warmup 0 $NB" \
  tests
