#!/bin/bash
# Stop the processes started by system_start.sh (by their recorded PIDs only).
cd "$(dirname "$0")/.."
for name in registrar broker; do
  if [[ -f .aiko/$name.pid ]]; then
    kill "$(cat .aiko/$name.pid)" 2>/dev/null || true
    rm -f .aiko/$name.pid
  fi
done
