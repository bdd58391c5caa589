#!/bin/bash
# weight-gradient knobs re-checked after the asm LDS-DMA change: split multiplier, weight lane
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_env.sh DVIE_WG_SPLITS 2 1 ${1:-r04al}/ab_splits || exit 1
bash tools/ab_env.sh DVIE_WGRAD_LANE 0 1 ${1:-r04al}/ab_lane || exit 1
