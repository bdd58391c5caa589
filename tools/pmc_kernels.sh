#!/bin/bash
# PMC counters of the dominant conv kernels on the bench command: one rocprofv3 pass per
# counter group (SQ / TCC limits per pass; FETCH_SIZE and WRITE_SIZE cannot share one),
# plus one kernel-trace pass for durations.  Report: tools/pmc_kernels_report.py.
# usage (via gpurun): [PMC_RX=<kernel regex>] [PMC_CMD=<command>] bash tools/pmc_kernels.sh <tag>
set -o pipefail
tag=${1:-pmck}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
rx=${PMC_RX:-"conv_halo_kernel|conv_ws_kernel|conv_strip_kernel|conv_nk_kernel|conv1x1_kernel|conv1x1_persist_kernel|wgrad_halo_kernel|wgrad_wide_kernel|conv_igemm_kernel|wgrad_kernel"}
cmd=${PMC_CMD:-"python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-steps 0 --graph 0"}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$rx" --output-format csv -d $out/p$i -o run -- $cmd > $out/p$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 $out/p$i.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- $cmd > $out/trace.log 2>&1 \
  || { echo "trace pass failed"; tail -20 $out/trace.log; exit 1; }
rm -f $out/trace/*kernel_trace.csv
python3 tools/pmc_kernels_report.py $out > $out/report.txt && cat $out/report.txt
