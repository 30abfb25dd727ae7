#!/bin/bash
# Print every message in this namespace (reference scripts/mqtt_sub_all.sh).
cd "$(dirname "$0")/.."
python3 -m aiko_services_amd.tools.mqtt sub "${AIKO_NAMESPACE:-aiko}/#"
