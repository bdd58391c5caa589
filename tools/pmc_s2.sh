#!/bin/bash
# PMC passes on one stride-2 forward conv shape (tools/conv_micro.py), conv_s2 kernel only,
# plus the device's counter list.  usage (via gpurun): bash tools/pmc_s2.sh <tag> <conv_micro args...>
set -o pipefail
tag=$1; shift
out=gpurun_out/pmc/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > $out/avail.txt 2>&1 || echo "list failed"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "TA_BUSY_avr TA_TA_BUSY_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "conv_s2|conv_igemm" --output-format csv -d $out -o p$i -- python3 tools/conv_micro.py "$@" > $out/p$i.log 2>&1 || echo "pass $i ($grp) failed"
done
find $out -name '*counter_collection.csv'
echo ok
