#!/bin/bash
# round-3 session Q: WRITE_SIZE calibration on the trace kernel's store width, VALU lane
# utilisation of the binary and 4-wide (RT_WIDE) C2 walks (1200x800x100), C4 phase shares at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/rust-ray-tracing-in-a-weekend_amd/lib
NB="--no-cpu-baseline --no-count"
SQA="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P="timeout -s KILL 200 rocprofv3 --output-format csv"
scripts/gpu_session.sh \
  "200:r03q_write_calib:export TMPDIR=/tmp; $P --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r03q_write_calib -o w -- scripts/calib/write_calib" \
  "300:r03q_sqa_bin:export TMPDIR=/tmp; $P --pmc $SQA -d gpurun_out/r03q_sqa_bin -o s -- python3 bench.py --steps 2 --warmup 1 --spp 100 $NB" \
  "300:r03q_sqa_w4:export TMPDIR=/tmp RT_LIB_PATH=$L/librtiow_exp_w4.so; $P --pmc $SQA -d gpurun_out/r03q_sqa_w4 -o s -- python3 bench.py --steps 2 --warmup 1 --spp 100 $NB" \
  "300:r03q_phases_c4:python scripts/phases.py --scene 7 --width 1920 --height 1080 --spp 8"
