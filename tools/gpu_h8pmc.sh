#!/bin/bash
# conv_h8 vs conv_halo<2,2,4,3,3> on HRNet's 128- and 256-channel 3x3 shapes: timing, then PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-h8pmc}; mkdir -p $out
timeout -k 10 200 python -u tools/conv_tune.py -3,4,-3,4 20 '128->128|256->256' > $out/tune.txt 2>&1 || { tail -20 $out/tune.txt; exit 1; }
cat $out/tune.txt
PMC_RX="conv_h8_kernel|conv_halo_kernel" PMC_CMD="python3 tools/conv_tune.py -3,4 5 128->128|256->256" bash tools/pmc_kernels.sh ${1:-h8pmc}/pmc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k warp > $out/pytest_warp.log 2>&1 \
  || { tail -30 $out/pytest_warp.log; exit 1; }
tail -2 $out/pytest_warp.log
for g in 8192 2048 1024 512; do
  DVIE_WARP_FWD_GRID=$g timeout -k 10 120 python -u tools/warp_micro.py --reps 50 > $out/warp_$g.txt 2>&1 || { tail $out/warp_$g.txt; exit 1; }
  echo "grid cap $g"; grep -i "fwd" $out/warp_$g.txt
done
