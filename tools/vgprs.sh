#!/bin/bash
# VGPR / AGPR / spill / occupancy per kernel of one HIP source (compiler resource remarks)
# usage: bash tools/vgprs.sh deep_video_interpolation_extrapolation_amd/csrc/conv_halo.hip [filter]
f=$1; pat=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c "$f" -o /tmp/vgprs.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | awk '/Function Name/{n=$3} /^VGPRs:/{v=$2} /^AGPRs:/{a=$2} /VGPRs Spill/{s=$3} /Occupancy/{o=$3; print n, "vgpr="v, "agpr="a, "spill="s, "occ="o}' |
  c++filt | grep -E "$pat"
