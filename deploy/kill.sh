#!/bin/bash
# Stop the processes started by run_exp.sh: exactly the recorded PIDs, host by host
# (the reference's kill.sh runs `pkill -f trainer.py` on every host, which also
# hits unrelated processes whose command line matches).
set -uo pipefail
SSH=${SSH:-ssh}
PIDS=${1:-run_exp.pids}
while read -r host pid; do
  [ -z "$host" ] && continue
  echo "stopping $pid on $host"
  $SSH "$host" "kill $pid" < /dev/null || true
done < "$PIDS"
