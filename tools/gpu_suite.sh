#!/bin/bash
# Runs GPU steps in order; each under its own time limit.  A pytest failure (rc 1) does not
# stop the suite; a timeout / abort / segfault / fault (any other non-zero) stops it.
# usage: tools/gpu_suite.sh NAME:SECONDS:CMD [NAME:SECONDS:CMD ...]
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -4 "gpurun_out/$name.log"
  case $rc in
    0|1|5) ;;
    *) echo "stopping: $name exited $rc"; exit $rc ;;
  esac
done
