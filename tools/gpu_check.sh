#!/bin/bash
# One GPU session: tests, smoke, bench. Each GPU step has its own time limit;
# a crash/abort/timeout (status >= 124 or signal) ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "fatal step $name ($rc), stopping" >&2; exit $rc; fi
  return $rc
}
