#!/bin/bash
# bench.py (default workload) with its per-op table, then a rocprofv3 kernel-trace summary of
# the same command; usage (via gpurun): bash tools/gpu_bench_ops.sh <tag> [bench args...]
set -o pipefail
tag=${1:-bench}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 420 python -u bench.py --ops-out $out/ops.txt "$@" > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 "$@" > $out/bench_prof.json 2> $out/bench_prof.err || { echo "rocprof failed"; tail -20 $out/bench_prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
rm -f $out/prof/*/*kernel_trace.csv
head -15 $out/kernel_stats.csv | cut -c1-200
