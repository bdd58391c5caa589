#!/bin/bash
# Same-box A/B of the bench step under two values of one environment knob.
# usage (via gpurun): bash tools/ab_env.sh VAR A B [tag]
set -o pipefail
var=$1; va=$2; vb=$3; tag=${4:-ab_$1}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in $va $vb; do
    env $var=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0 \
      > gpurun_out/$tag/b_${v}_$r.json 2> gpurun_out/$tag/b_${v}_$r.err || { tail -20 gpurun_out/$tag/b_${v}_$r.err; exit 1; }
    echo "$var=$v run $r $(grep -o '"value": [0-9.]*' gpurun_out/$tag/b_${v}_$r.json)"
  done
done
