#!/bin/bash
# SQ counter passes over the bench workload (one rocprofv3 --pmc pass per group, no traces).
# usage: BENCH_ARGS="..." scripts/sq_passes.sh OUTDIR "C1 C2 C3 C4" "C5 ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --no-count"}
i=0
for group in "$@"; do
    i=$((i + 1))
    timeout -k 10 200 rocprofv3 --pmc $group --output-format csv -d $OUT/p$i -o p$i -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || exit 3
done
find $OUT -name "*counter_collection.csv"
