#!/bin/bash
# Build the native extensions here (incremental), then run a command on the GPU box.
# usage: scripts/gpu.sh <timeout-seconds> '<command>'
set -e
cd "$(dirname "$0")/.."
python -c "from distributed_amd import _build; _build.build(False)"
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
