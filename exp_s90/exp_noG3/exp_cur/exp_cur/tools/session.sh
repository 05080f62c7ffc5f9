#!/bin/bash
# One GPU-box session: STEPS are "name|limit|command" lines read from the file given as $2; output under
# gpurun_out/$1/<name>.log.  Test failures (exit 1) continue; any other non-zero exit (fault, abort,
# timeout) stops the session there.
O=gpurun_out/$1; mkdir -p "$O"; export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
while IFS='|' read -r name lim cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue ;; esac
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name ended with $rc"; tail -20 "$O/$name.log"; exit $rc; fi
done < "$2"
echo done
