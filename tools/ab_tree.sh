#!/bin/bash
# Same-box A/B of two trees: an older commit checked out and built in _ab_old (git worktree add
# _ab_old <commit>; make -C _ab_old/deep_video_interpolation_extrapolation_amd/csrc) and the current tree.
# usage (via gpurun): bash tools/ab_tree.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abtree
for r in 1 2; do
  for t in old new; do
    d=.; [ $t = old ] && d=_ab_old
    (cd $d && timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0) > gpurun_out/abtree/b_${t}_$r.json 2> gpurun_out/abtree/b_${t}_$r.err || { tail -5 gpurun_out/abtree/b_${t}_$r.err; exit 1; }
    echo "$t run $r $(grep -o '"value": [0-9.]*' gpurun_out/abtree/b_${t}_$r.json)"
  done
done
