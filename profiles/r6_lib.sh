#!/bin/bash
# Shared by the round-6 GPU scripts: run one step under its own time limit; a test failure (rc 1)
# is recorded and the script goes on, a timeout / abort / fault (rc >= 124) ends the script.
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[r6] $name: $*"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "[r6] $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "[r6] stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
