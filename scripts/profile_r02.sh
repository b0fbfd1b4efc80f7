#!/bin/bash
# rocprofv3 passes for one bench workload (run on the GPU box from the repo root):
#   kt     kernel trace + stats (per-kernel durations; must agree with bench.py's HIP events)
#   sqa    PMC: VALU issue / lane counters + GRBM_GUI_ACTIVE (clock)
#   sqb    PMC: VALU instruction classes (the mix the roofline prices)
#   fetch  PMC: FETCH_SIZE (own pass: TCC slots)
#   write  PMC: WRITE_SIZE (own pass)
# Each pass in its own run and time limit (MI355X_MICROARCH.md §rocprofv3 PMC slots); stop at
# the first failure. usage: PROF_DIR=name BENCH_ARGS="..." scripts/profile_r02.sh
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_DIR:-prof}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --no-count"}
LIM=${PASS_LIMIT:-240}
SQA="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
SQC="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
timeout -k 10 $LIM rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
timeout -s KILL $LIM rocprofv3 --pmc $SQA --output-format csv -d $OUT/sqa -o sqa -- python3 bench.py $ARGS > $OUT/sqa.log 2>&1
timeout -s KILL $LIM rocprofv3 --pmc $SQB --output-format csv -d $OUT/sqb -o sqb -- python3 bench.py $ARGS > $OUT/sqb.log 2>&1
timeout -s KILL $LIM rocprofv3 --pmc $SQC --output-format csv -d $OUT/sqc -o sqc -- python3 bench.py $ARGS > $OUT/sqc.log 2>&1
timeout -s KILL $LIM rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL $LIM rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 bench.py $ARGS > $OUT/write.log 2>&1
find $OUT -name "*.csv" | head -50
