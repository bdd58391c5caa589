#!/bin/bash
# Kernel times of one conv shape (tools/conv_micro.py) under several env settings, one
# rocprofv3 kernel-trace run each.  usage (via gpurun):
#   bash tools/s2_ab.sh <tag> "<ENV=..>" "<ENV=..>" ... -- <conv_micro args...>
set -o pipefail
tag=$1; shift
envs=()
while [ "$1" != "--" ]; do envs+=("$1"); shift; done
shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for e in "${envs[@]}"; do
  i=$((i+1))
  ( export $e; timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/r$i -o k -- python3 tools/conv_micro.py "$@" > $out/r$i.log 2>&1 ) || { echo "run $i ($e) failed"; tail -5 $out/r$i.log; exit 1; }
  f=$(find $out/r$i -name '*kernel_stats.csv')
  echo "== $e"; grep -E "conv_s2|conv_igemm|conv1x1|wgrad" $f | cut -d, -f1-4 || true
  rm -f $out/r$i/*/*kernel_trace.csv
done
