#!/bin/bash
# Run GPU steps in order; stop at the first step that ends in anything other
# than success or an ordinary test failure (exit 1): a fault, abort, segfault
# or time-out ends the session (no further GPU work in this call).
#   tools/gpu_session.sh "name:timeout:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${to}s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping after $name (rc=$rc)"
    exit $rc
  fi
done
