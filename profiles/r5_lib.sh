#!/bin/bash
# Shared by the round-5 GPU scripts: run one step under its own time limit; a test failure (rc 1)
# is recorded and the script goes on, a timeout / abort / fault (rc >= 124) ends the script.
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[r5] $name: $*"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "[r5] $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "[r5] stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYT=(python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider)
