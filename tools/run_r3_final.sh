#!/bin/bash
# round 3: GPU suite + default bench line + rocprofv3 profile at the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r3d}
TAG=$TAG bash tools/run_r3_suite.sh || exit 1
TAG=$TAG bash tools/run_r3_bench_prof.sh || exit 1
