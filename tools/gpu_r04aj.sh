#!/bin/bash
# weight-gradient tile walk without divisions (incremental tile position, constant-divisor
# halo-piece mapping): timing A/B against the committed build + PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04aj}; mkdir -p $out
cp deep_video_interpolation_extrapolation_amd/libdvie.so /tmp/libdvie_base.so
cp tools/probe/libdvie_new7.so deep_video_interpolation_extrapolation_amd/libdvie.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wgrad.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for r in 1 2; do
  for l in base new; do
    if [ $l = base ]; then L=/tmp/libdvie_base.so; else L=tools/probe/libdvie_new7.so; fi
    DVIE_TOOL_LIB=$L timeout -k 10 200 python -u tools/wgrad_tune.py 10 '3x3' > $out/wg_${l}_$r.txt 2>&1 || { tail $out/wg_${l}_$r.txt; exit 1; }
    echo "$l $r"; grep "3x3" $out/wg_${l}_$r.txt | cut -c1-75
  done
done
PMC_RX="wgrad_halo_kernel" PMC_CMD="python3 tools/wgrad_tune.py 5 3x3 64->64" bash tools/pmc_kernels.sh ${1:-r04aj}/wg || exit 1
