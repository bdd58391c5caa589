#!/bin/bash
# r04: captured vs eager step on C2 and C5, executor lanes on / off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04v}; mkdir -p $out
for g in 1 0; do
  for l in 1 0; do
    DVIE_OP_LANES=$l timeout -k 10 300 python -u bench.py --graph $g --no-cpu-baseline --profile-steps 0 > $out/c2_g${g}_l$l.json 2> $out/c2_g${g}_l$l.err || { echo "c2 failed"; tail -20 $out/c2_g${g}_l$l.err; exit 1; }
    python3 -c "import json;d=json.load(open('$out/c2_g${g}_l$l.json'));print('c2 graph=$g lanes=$l', d['value'], d['ms_per_step'], d['eager_ms_per_step'])"
  done
done
for l in 0 1; do
  DVIE_OP_LANES=$l timeout -k 10 500 python -u bench.py --workload c5 --no-cpu-baseline --profile-steps 0 > $out/c5_l$l.json 2> $out/c5_l$l.err || { echo "c5 failed"; tail -20 $out/c5_l$l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/c5_l$l.json'));print('c5 lanes=$l', d['value'], d['ms_per_step'], d['eager_ms_per_step'])"
done
