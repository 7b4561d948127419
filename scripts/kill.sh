#!/bin/bash
# Stop the processes this directory's launchers started (reference scripts/kill.sh, which
# killed every python3 process on the machine by name). Only the PIDs recorded in .drn_pids
# (and their process groups) are signalled -- never a name pattern.
PIDFILE=${1:-.drn_pids}
[ -f "$PIDFILE" ] || { echo "no $PIDFILE here"; exit 0; }
while read -r pid; do
  [ -n "$pid" ] || continue
  if kill -0 "$pid" 2>/dev/null; then
    kill -TERM -- "-$pid" 2>/dev/null || kill -TERM "$pid" 2>/dev/null
  fi
done < "$PIDFILE"
sleep "${GRACE:-5}"
while read -r pid; do
  [ -n "$pid" ] || continue
  kill -0 "$pid" 2>/dev/null && { kill -KILL -- "-$pid" 2>/dev/null || kill -KILL "$pid" 2>/dev/null; }
done < "$PIDFILE"
rm -f "$PIDFILE"
