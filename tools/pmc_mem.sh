#!/bin/bash
# Vector-memory pipeline counters (TA address unit, TCP L1, UTCL1 translation) per kernel:
# one rocprofv3 pass per group, within gfx950's per-pass limits (TA 2, TCP 4, GRBM 2).
# usage (via gpurun): PMC_RX=<kernel regex> PMC_CMD=<command> bash tools/pmc_mem.sh <tag>
# report: python3 tools/pmc_mem_report.py gpurun_out/<tag>
set -o pipefail
tag=${1:-pmcm}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
rx=${PMC_RX:?kernel regex}
cmd=${PMC_CMD:?command}
i=0
for grp in "TA_BUSY_avr TA_BUFFER_TOTAL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_REQUEST_sum" \
           "TA_BUFFER_COALESCED_READ_CYCLES_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum SQ_WAVES SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$rx" --output-format csv -d $out/p$i -o run -- $cmd > $out/p$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 $out/p$i.log; exit 1; }
done
python3 tools/pmc_mem_report.py $out > $out/report.txt && cat $out/report.txt
