#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-tim} bash tools/timing.sh
rc=$?
cat gpurun_out/${TAG:-tim}/timing.txt
exit $rc
