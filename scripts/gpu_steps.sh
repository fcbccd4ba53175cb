#!/bin/bash
# Run a list of GPU steps "name|timeout|command" from the file given as $1 (one
# per line), each under its own time limit, output in gpurun_out/<name>.log.
# A test failure does not stop the list; a crash-class exit (timeout, abort,
# segfault, kill) does -- nothing more touches the GPU after that.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTD=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
while IFS='|' read -r name tmo cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  echo "[gpu_steps] $name (limit ${tmo}s): $cmd"
  ( cd "$ROOTD" && eval "timeout -k 10 $tmo env $cmd" ) > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "[gpu_steps] crash-class exit; stopping"; exit $rc;; esac
done < "$1"
exit 0
