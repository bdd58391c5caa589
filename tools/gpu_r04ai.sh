#!/bin/bash
# PMC counters of the 3x3 weight gradient (halo kernel, asm DMA) and the 64-channel strip conv
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04ai}; mkdir -p $out
PMC_RX="wgrad_halo_kernel" PMC_CMD="python3 tools/wgrad_tune.py 5 3x3 64->64" bash tools/pmc_kernels.sh ${1:-r04ai}/wg || exit 1
PMC_RX="conv_strip_kernel" PMC_CMD="python3 tools/conv_tune.py -3 5 3x3 64->64" bash tools/pmc_kernels.sh ${1:-r04ai}/strip || exit 1
