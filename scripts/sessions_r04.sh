#!/bin/bash
# Round-4 GPU sessions, one case each (run through gpurun from the repo root):
#   /usr/local/graft/bin/gpurun -- scripts/sessions_r04.sh <letter>
# Each writes gpurun_out/r04<letter>_*.log; the logs kept under profiles/ name their session.
# Steps go through scripts/gpu_session.sh (each under its own time limit; a fault stops the session).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=rust-ray-tracing-in-a-weekend_amd/lib
NB="--no-cpu-baseline --no-count"
case "$1" in
a)
    # round-4 session A: the byte-exact output / RCCL-branch / empty-shard build — GPU tests, smoke, default bench
    PREFIX=r04a_ scripts/gpu_session.sh tests smoke bench
    ;;
*)
    echo "unknown session: $1" >&2; exit 2 ;;
esac
