#!/bin/bash
# Runs GPU steps in order, each under its own time limit. A step that exits 0 or 1
# (tests passed / some assertions failed) lets the next step run; anything else
# (fault, abort, segfault, timeout) stops the script.
# usage: scripts/gpu_steps.sh "<seconds>:<name>:<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
    secs="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== $name (limit ${secs}s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name exit $rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (exit $rc)"; exit $rc; fi
done
