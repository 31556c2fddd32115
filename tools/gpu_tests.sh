#!/bin/bash
# tools/gpu_tests.sh TAG [pytest args...] -- run on the GPU box (via gpurun): the full `pytest -m gpu` suite
# (or the given selection) with the tree's revision as the log's first line.  The revision comes from
# REVISION, written by tools/stamp_revision.sh in the build container just before the gpurun call (the
# box gets no .git).  Log: gpurun_out/gputest_TAG.log (copied to profiles/ when kept).
set -u
TAG=${1:-run}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
LOG=$R/gpurun_out/gputest_$TAG.log
mkdir -p "$R/gpurun_out"
{ echo "revision: $(cat "$R/REVISION" 2>/dev/null || echo unknown)"; echo "host: $(hostname) date: $(date -u +%FT%TZ)"; } > "$LOG"
cd "$R"
export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests)
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${ARGS[@]}" >> "$LOG" 2>&1
rc=$?
tail -3 "$LOG"
exit $rc
