#!/bin/bash
# VALU calibration on the GPU box (scripts/calib/valu_calib.hip, built here with hipcc):
# in-binary timing of every class in three modes, then PMC passes over the saturated runs
# (what SQ_INSTS_VALU and the class counters report for instructions of known class and
# count). usage: scripts/calib_r02.sh OUTDIR
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-calib}
mkdir -p $OUT
B=scripts/calib/valu_calib
timeout -k 10 120 $B all sat,one,lat 4000 > $OUT/timing.jsonl
SQA="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
SQC="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --pmc $SQA --output-format csv -d $OUT/sqa -o sqa -- $B all sat 1000 > $OUT/sqa.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $SQB --output-format csv -d $OUT/sqb -o sqb -- $B all sat 1000 > $OUT/sqb.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $SQC --output-format csv -d $OUT/sqc -o sqc -- $B all sat 1000 > $OUT/sqc.log 2>&1
find $OUT -name "*.csv"
