#!/bin/bash
# warp forward A/B: non-temporal stores / loads, grid caps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-warpnt}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k warp > $out/pytest_warp.log 2>&1 \
  || { tail -30 $out/pytest_warp.log; exit 1; }
tail -1 $out/pytest_warp.log
for r in 1 2; do
for v in "0 0" "1 0" "2 0" "0 16384" "1 16384" "0 4096"; do
  set -- $v
  DVIE_WARP_NT=$1 DVIE_WARP_FWD_GRID=$2 timeout -k 10 120 python -u tools/warp_micro.py --reps 50 > $out/w_$1_$2_$r.txt 2>&1 || { tail $out/w_$1_$2_$r.txt; exit 1; }
  echo "nt=$1 grid=$2 run $r: $(grep fwd $out/w_$1_$2_$r.txt | tr '\n' ' ')"
done
done
timeout -k 10 120 python -u tools/probe/store_probe.py > $out/store_probe.txt 2>&1 || { tail $out/store_probe.txt; exit 1; }
cat $out/store_probe.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_epilogue.py -k "coalesced or 1x1 or 64-256 or conv_epilogue_operands" > $out/pytest_ce.log 2>&1 \
  || { tail -30 $out/pytest_ce.log; exit 1; }
tail -1 $out/pytest_ce.log
bash tools/ab_env.sh DVIE_1X1_CE 1 0 ${1:-warpnt}/ab_ce || exit 1
