#!/bin/bash
# End-of-round pass 2: the BASELINE config-5 workload line (bench.py --workload c5, per-op
# table), the conv family's HBM traffic from PMC counters (the bench's roofline.traffic
# source) and the per-kernel counter report, on the same tree as tools/gpu_round.sh.
# usage (via gpurun): bash tools/gpu_final2.sh <tag>
set -o pipefail
tag=${1:-final2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u bench.py --workload c5 --ops-out $out/ops_c5.txt > $out/bench_c5.json 2> $out/bench_c5.err \
  || { echo "c5 bench failed"; tail -20 $out/bench_c5.err; exit 1; }
cat $out/bench_c5.json
bash tools/pmc_bench.sh $tag/pmc > /dev/null || exit 1
tail -5 $out/pmc/traffic.txt
PMC_RX="head3_bwd_kernel|segenc_fwd_kernel|segenc_bwd_kernel|conv_narrow_kernel|conv_h8_kernel|conv_halo_kernel|conv_ws_kernel|conv_strip_kernel|conv_nk_kernel|conv1x1_kernel|conv1x1_persist_kernel|conv1x1_ring_kernel|conv_s2_kernel|wgrad_halo_kernel|wgrad_kernel|wgrad_wide_kernel" \
  bash tools/pmc_kernels.sh $tag/pmck > /dev/null || exit 1
python3 tools/pmc_kernels_report.py $out/pmck > $out/pmc_kernels_report.txt && head -30 $out/pmc_kernels_report.txt
echo done
