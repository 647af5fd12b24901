#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/.
#   tools/gpu_steps.sh "<name>|<seconds>|<command>" ...
# A step that fails normally (e.g. a test failure, exit 1) does not stop the
# next one; a time limit (124/137), an abort (134) or a segfault (139) ends the
# script there, so nothing more touches the GPU after a fault or a hang.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  mkdir -p "$(dirname "gpurun_out/$name.log")"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc after $(( $(date +%s) - start ))s"
  tail -n 5 "gpurun_out/$name.log"
  case $rc in
    124|137|134|139) echo "=== fatal exit $rc: stopping"; exit $rc ;;
  esac
done
