#!/bin/bash
# HBM traffic of the bench's conv kernels from PMC counters: one rocprofv3 pass per TCC
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), on the same
# bench command, restricted to the conv forward / data-gradient kernels.
# usage (via gpurun): bash tools/pmc_bench.sh <tag>
set -o pipefail
tag=${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
rx="head3_bwd_kernel|segenc_fwd_kernel|segenc_bwd_kernel|conv_narrow_kernel|conv_h8_kernel|conv_halo_kernel|conv_ws_kernel|conv_strip_kernel|conv_nk_kernel|conv1x1_kernel|conv1x1_persist_kernel|conv1x1_ring_kernel|conv_s2_kernel|conv_igemm_kernel|wgrad_halo_kernel|wgrad_kernel|wgrad_wide_kernel"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "$rx" --output-format csv -d $out/$c -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-steps 0 --graph 0 > $out/$c.log 2>&1 \
    || { echo "pmc pass $c failed"; tail -20 $out/$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $out > $out/traffic.txt && cat $out/traffic.txt
