#!/bin/bash
# Warp parity tests, then the warp micro-benchmark twice under each value of an A/B knob
# (AB_VAR, values AB_VALS; the printed gradient digests must agree where the backward has
# no far-corner atomics), then rocprofv3 kernel stats of the micro run.
# usage (via gpurun): bash tools/gpu_warp.sh <tag>
set -o pipefail
tag=${1:-warp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k warp -x -v --timeout 120 --timeout-method thread > $out/pytest_warp.log 2>&1 || { echo "warp tests failed"; grep -E "FAIL|Error|assert" $out/pytest_warp.log | head -20; tail -30 $out/pytest_warp.log; exit 1; }
tail -2 $out/pytest_warp.log
var=${AB_VAR:-DVIE_WARP_WIN}
for m in ${AB_VALS:-4 3 4 3}; do
  env $var=$m timeout -k 10 120 python -u tools/warp_micro.py --reps 50 > $out/micro_$var$m.txt 2>&1 || { echo "micro $m failed"; tail $out/micro_$var$m.txt; exit 1; }
  echo "$var=$m"; grep -v amdgpu.ids $out/micro_$var$m.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o warp -- python3 tools/warp_micro.py --reps 20 > $out/prof.log 2>&1 || { echo "rocprof failed"; tail $out/prof.log; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
rm -f $out/prof/*/*kernel_trace.csv
cut -d, -f1-8 $out/kernel_stats.csv | head -12
