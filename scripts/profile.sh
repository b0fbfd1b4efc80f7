#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root).
#   1. kernel trace + stats      (per-kernel durations; must agree with bench.py's HIP events)
#   2. PMC FETCH_SIZE            (own pass: TCC slots)
#   3. PMC WRITE_SIZE            (own pass)
#   4. PMC SQ counters           (waves, VALU/SALU/VMEM instruction mix, busy cycles)
# Each pass under its own time limit; stop at the first failure.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_DIR:-prof}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --no-count"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc ${SQ_PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE} --output-format csv -d $OUT/sq -o sq -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || echo "SQ pass failed (counter names?)"
find $OUT -name "*.csv" | head -50
