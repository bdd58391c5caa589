#!/bin/bash
# conv / pointwise knobs re-checked on the final tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_env.sh DVIE_CONV_STRIP 1 2 ${1:-r04an}/ab_strip || exit 1
bash tools/ab_env.sh DVIE_1X1_PERSIST 0 1 ${1:-r04an}/ab_persist || exit 1
bash tools/ab_env.sh DVIE_EW_FUSE2 0 1 ${1:-r04an}/ab_fuse2 || exit 1
