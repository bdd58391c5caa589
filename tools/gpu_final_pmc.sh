#!/bin/bash
# End-of-round counters on the bench command: HBM traffic of the conv family (the bench's
# `roofline.traffic` source) and the per-kernel PMC report, plus the VGG deep-block tile sweep.
# usage (via gpurun): bash tools/gpu_final_pmc.sh <tag>
set -o pipefail
tag=${1:-r06pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 240 python3 -u tools/conv_tune.py -3,1,5,4,0,3 20 'b8|b16' > gpurun_out/$tag/vgg_tune.txt 2>&1 \
  || { echo "tune failed"; tail -20 gpurun_out/$tag/vgg_tune.txt; exit 1; }
cat gpurun_out/$tag/vgg_tune.txt
bash tools/pmc_bench.sh $tag/pmc > /dev/null || exit 1
tail -5 gpurun_out/$tag/pmc/traffic.txt
PMC_RX="head3_bwd_kernel|segenc_bwd_kernel|conv_narrow_kernel|conv_h8_kernel|conv_halo_kernel|conv_ws_kernel|conv_strip_kernel|conv_nk_kernel|conv1x1_kernel|conv1x1_persist_kernel|conv1x1_ring_kernel|conv_s2_kernel|wgrad_halo_kernel|wgrad_kernel|wgrad_wide_kernel" \
  bash tools/pmc_kernels.sh $tag/pmck > /dev/null || exit 1
head -30 gpurun_out/$tag/pmck/report.txt
