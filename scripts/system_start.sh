#!/bin/bash
# Start the aiko control plane on this host: in-repo MQTT broker (if AIKO_MQTT_HOST is local),
# registrar, and optionally the dashboard (reference scripts/system_start.sh).
#   scripts/system_start.sh [--no-dashboard]
set -e
cd "$(dirname "$0")/.."
export AIKO_MQTT_HOST=${AIKO_MQTT_HOST:-127.0.0.1}
export AIKO_MQTT_PORT=${AIKO_MQTT_PORT:-1883}
mkdir -p .aiko
if [[ "$AIKO_MQTT_HOST" == "127.0.0.1" || "$AIKO_MQTT_HOST" == "localhost" ]]; then
  python3 -m aiko_services_amd.tools.mqtt broker --port "$AIKO_MQTT_PORT" > .aiko/broker.log 2>&1 &
  echo $! > .aiko/broker.pid
  sleep 0.5
fi
python3 -m aiko_services_amd.tools.registrar > .aiko/registrar.log 2>&1 &
echo $! > .aiko/registrar.pid
sleep 0.5
if [[ "$1" != "--no-dashboard" ]]; then
  python3 -m aiko_services_amd.tools.dashboard
fi
