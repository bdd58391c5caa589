#!/bin/bash
# Price op kinds in the eager step: the timing-only library (-DDVIE_TIMING_DBG, results wrong)
# with DVIE_SKIP_KINDS = bit masks of dvie_op kinds left out (include/dvie.h DVIE_OP_*).
# usage (via gpurun): bash tools/skip_ab.sh TAG MASK...
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
pkg=deep_video_interpolation_extrapolation_amd/libdvie.so
cp $pkg $out/orig.so
trap 'cp $out/orig.so $pkg' EXIT
cp tools/probe/libdvie_tdbg.so $pkg || exit 1
for m in "$@"; do
  DVIE_SKIP_KINDS=$m timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0 > $out/b_$m.json 2> $out/b_$m.err || { tail -5 $out/b_$m.err; exit 1; }
  echo "skip mask $m: $(python3 -c "import json;d=json.load(open('$out/b_$m.json'));print(d['value'], d['ms_per_step'])")"
done
