#!/bin/bash
# LDS-DMA through inline asm (no compiler vmcnt(0) before the LDS reads) in the weight-gradient
# and fused head-backward kernels; deep-pipelined 3x3 weight gradient; same-box lib A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04ae}; mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wgrad.py tests/test_gpu_head3.py \
  tests/test_gpu_parity.py tests/test_gpu_train.py::test_inter_step_matches_reference tests/test_gpu_configs.py::test_c2_bf16_step_256x512_b8_quality \
  > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for v in 1 0; do
  DVIE_WG_DEEP=$v timeout -k 10 200 python -u tools/wgrad_tune.py 10 '3x3 64->64|3x3 128->128|3x3 256->256|1x1' > $out/wg_deep_$v.txt 2>&1 || { tail $out/wg_deep_$v.txt; exit 1; }
  echo "deep=$v"; grep -v "^$" $out/wg_deep_$v.txt | tail -7
done
DVIE_TOOL_LIB=tools/probe/libdvie_r04z.so timeout -k 10 200 python -u tools/wgrad_tune.py 10 '3x3 64->64|3x3 128->128|3x3 256->256|1x1' > $out/wg_r04z.txt 2>&1 || { tail $out/wg_r04z.txt; exit 1; }
echo "r04z lib"; grep -v "^$" $out/wg_r04z.txt | tail -7
cp deep_video_interpolation_extrapolation_amd/libdvie.so /tmp/libdvie_cur.so && bash tools/ab_lib.sh tools/probe/libdvie_r04z.so /tmp/libdvie_cur.so ${1:-r04ae}/ab_lib || exit 1
