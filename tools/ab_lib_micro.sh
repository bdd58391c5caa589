#!/bin/bash
# Same-box kernel times of one conv shape (tools/conv_micro.py) under two builds of libdvie.so.
# usage (via gpurun): bash tools/ab_lib_micro.sh LIB_A LIB_B TAG REGEX -- <conv_micro args...>
set -o pipefail
la=$1; lb=$2; tag=$3; rx=$4; shift 4; [ "$1" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
pkg=deep_video_interpolation_extrapolation_amd/libdvie.so
cp $pkg $out/orig.so
# restore the package library however the script ends (outer timeout / SIGKILL of a child included)
trap 'cp $out/orig.so $pkg' EXIT
for v in a b a b; do
  lib=$([ $v = a ] && echo $la || echo $lb)
  cp "$lib" $pkg
  rm -rf $out/r_$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/r_$v -o k -- python3 tools/conv_micro.py "$@" > $out/r_$v.log 2>&1 || { echo "run $v failed"; tail -5 $out/r_$v.log; cp $out/orig.so $pkg; exit 1; }
  f=$(find $out/r_$v -name '*kernel_stats.csv')
  echo "== $v $(basename $lib)"; grep -E "$rx" $f | awk -F'",' '{print $1"\"", $2}' | cut -c1-160
  rm -f $out/r_$v/*/*kernel_trace.csv
done
cp $out/orig.so $pkg
