#!/bin/bash
# warp forward A/B: non-temporal stores / loads, grid caps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-warpnt}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k warp > $out/pytest_warp.log 2>&1 \
  || { tail -30 $out/pytest_warp.log; exit 1; }
tail -1 $out/pytest_warp.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_epilogue.py -k "coalesced or transposed or conv_epilogue_operands or h8_modes" > $out/pytest_ce.log 2>&1 \
  || { tail -30 $out/pytest_ce.log; exit 1; }
tail -1 $out/pytest_ce.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py::test_inter_step_matches_reference \
  tests/test_gpu_configs.py::test_c2_bf16_step_256x512_b8_quality tests/test_gpu_head3.py > $out/pytest_plan.log 2>&1 \
  || { tail -30 $out/pytest_plan.log; exit 1; }
tail -1 $out/pytest_plan.log
bash tools/ab_env.sh DVIE_1X1_CE 1 0 ${1:-warpnt}/ab_ce || exit 1
bash tools/ab_env.sh DVIE_H8_CE 1 0 ${1:-warpnt}/ab_h8ce || exit 1
for dbg in 0 8 16 32 56; do
  DVIE_TOOL_LIB=tools/probe/libdvie_timing.so DVIE_WG_DBG=$dbg timeout -k 10 200 python -u tools/wgrad_tune.py 10 '3x3 64->64|3x3 128->128|3x3 256->256' > $out/wg_dbg_$dbg.txt 2>&1 || { tail $out/wg_dbg_$dbg.txt; exit 1; }
  echo "wg dbg=$dbg"; grep -v "^$" $out/wg_dbg_$dbg.txt | tail -4
done
