#!/bin/bash
# Eager-step kernel census of the bench (tools/eager_census.py) and PMC HBM traffic of the
# conv / wgrad families on this tree (tools/pmc_bench.sh).  usage (via gpurun):
#   bash tools/gpu_census.sh <tag>
set -o pipefail
tag=${1:-census}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 420 python -u bench.py --ops-out $out/ops.txt > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'])"
for k in 2 6; do
  DVIE_OP_LANES=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/s$k -o run \
    -- python3 bench.py --steps $k --warmup 1 --no-cpu-baseline --profile-steps 0 > $out/s$k.log 2>&1 \
    || { echo "census run $k failed"; tail -20 $out/s$k.log; exit 1; }
  find $out/s$k -name '*kernel_stats.csv' -exec cp {} $out/stats_s$k.csv \;
  rm -f $out/s$k/*/*kernel_trace.csv
done
python3 tools/eager_census.py $out/stats_s2.csv $out/stats_s6.csv 4 > $out/eager_census.txt && cat $out/eager_census.txt
bash tools/pmc_bench.sh $tag/pmc
