#!/bin/bash
# Clear the retained registrar boot topic (a stale primary after a crash).
cd "$(dirname "$0")/.."
python3 -m aiko_services_amd.tools.mqtt reset
