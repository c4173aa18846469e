#!/bin/bash
# Run GPU steps in order on the gpurun box.  Each argument is "SECONDS|LOGNAME|COMMAND".
# Every step has its own time limit; a timeout / abort / segfault (124, 137, 134, 139)
# ends the session (nothing more touches the GPU); an ordinary failure (e.g. a
# failing test, exit 1) is recorded and the next step runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rc_all=0
for step in "$@"; do
  secs="${step%%|*}"; rest="${step#*|}"; log="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$log] $cmd (limit ${secs}s)"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log.log" 2>&1
  rc=$?
  echo "=== [$log] exit=$rc after $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$log.log"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  case $rc in
    124|137|134|139|143) echo "=== fatal exit code $rc: stopping GPU session"; exit $rc ;;
  esac
done
exit $rc_all
