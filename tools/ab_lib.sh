#!/bin/bash
# Same-box A/B of the bench step between two builds of libdvie.so (run on the GPU box, from the
# repo copy: each run copies its build over the package's libdvie.so first).
# usage (via gpurun): bash tools/ab_lib.sh LIB_A LIB_B [tag]
set -o pipefail
la=$1; lb=$2; tag=${3:-ab_lib}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$tag
pkg=deep_video_interpolation_extrapolation_amd/libdvie.so
cp $pkg gpurun_out/$tag/orig.so
trap 'cp gpurun_out/$tag/orig.so $pkg' EXIT  # the package library is restored however the script ends
for r in 1 2; do
  for v in a b; do
    if [ $v = a ]; then cp "$la" $pkg; else cp "$lb" $pkg; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0 \
      > gpurun_out/$tag/b_${v}_$r.json 2> gpurun_out/$tag/b_${v}_$r.err || { tail -20 gpurun_out/$tag/b_${v}_$r.err; exit 1; }
    echo "lib $v ($(basename $([ $v = a ] && echo $la || echo $lb))) run $r $(grep -o '"value": [0-9.]*' gpurun_out/$tag/b_${v}_$r.json)"
  done
done
