#!/bin/bash
# Same-box A/B of the round-5 tree (_ab_old: git worktree of c9b9152 with its own library) and
# the current tree (tools/ab_tree.sh, two runs each), then the current tree's warp objects.
# usage (via gpurun): bash tools/ab_round.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_tree.sh || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/abtree/b_new_2.json'));print('warp', d['warp']);print('warp1024', d['warp_1024x2048'])"
