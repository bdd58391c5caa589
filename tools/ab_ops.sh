#!/bin/bash
# Same-box A/B of two libdvie.so builds on the bench step WITH its per-op table (bench.py
# --ops-out): alternates the builds twice; the package library is restored however the script
# ends.  usage (via gpurun): bash tools/ab_ops.sh LIB_A LIB_B [tag]
set -o pipefail
la=$1; lb=$2; tag=${3:-ab_ops}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$tag
pkg=deep_video_interpolation_extrapolation_amd/libdvie.so
cp $pkg gpurun_out/$tag/orig.so
trap 'cp gpurun_out/$tag/orig.so $pkg' EXIT
for r in 1 2; do
  for v in a b; do
    if [ $v = a ]; then cp "$la" $pkg; else cp "$lb" $pkg; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --ops-out gpurun_out/$tag/ops_${v}_$r.txt \
      > gpurun_out/$tag/b_${v}_$r.json 2> gpurun_out/$tag/b_${v}_$r.err || { tail -20 gpurun_out/$tag/b_${v}_$r.err; exit 1; }
    echo "lib $v run $r $(grep -o '"value": [0-9.]*' gpurun_out/$tag/b_${v}_$r.json)"
  done
done
