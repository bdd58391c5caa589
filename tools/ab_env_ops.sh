#!/bin/bash
# Per-op tables of the bench step under several environment settings, same box.
# usage (via gpurun): bash tools/ab_env_ops.sh <tag> "VAR=a VAR2=b" "VAR=c" ...   ("-" = no extra env)
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
i=0
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --ops-out $out/ops_$i.txt > $out/b_$i.json 2> $out/b_$i.err || { echo "run $i ($e) failed"; tail -20 $out/b_$i.err; exit 1; }
  echo "$i [$e] $(python3 -c "import json;d=json.load(open('$out/b_$i.json'));print(d['value'], d['ms_per_step'], d['step_breakdown_ms'])")"
  i=$((i+1))
done
