#!/bin/bash
# timing build + per-phase row-kernel timings (tools/timing.sh), one box call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-tim} bash tools/timing.sh
