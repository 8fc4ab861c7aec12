#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
hipcc -O3 --offload-arch=gfx950 tools/flag_latency.hip -o /tmp/fl 2>/dev/null
timeout -k 5 60 /tmp/fl
