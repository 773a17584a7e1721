#!/bin/bash
# Run a command on the GPU box via gpurun; retry ONLY when gpurun reports that
# the box never ran it (status=transient / backing off: nothing charged).
# Usage: tools/gpu.sh <timeout_s> <logname> '<command>'
TO=$1; NAME=$2; CMD=$3
for i in 1 2 3 4 5 6; do
  timeout $((TO + 600)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > gpurun_out/$NAME.call.txt 2>&1
  rc=$?
  if grep -q -E "status=transient|backing off" gpurun_out/$NAME.call.txt; then
    sleep $((20 * i)); continue
  fi
  break
done
cat gpurun_out/$NAME.call.txt
exit $rc
