#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench line, rocprofv3 kernel-trace summary of bench.
# usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest_gpu.log; exit 1; }
  tail -3 $out/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
  tail -1 $out/smoke.log
fi
timeout -k 10 420 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
DVIE_OP_LANES=0 timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 --graph 0 > $out/bench_prof.json 2> $out/bench_prof.err || { echo "rocprof failed"; tail -20 $out/bench_prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec head -12 {} \;
if [ "$3" == "c5" ]; then  # BASELINE config 5 line with its per-op table
  timeout -k 10 600 python -u bench.py --workload c5 --ops-out $out/ops_c5.txt > $out/bench_c5.json 2> $out/bench_c5.err || { echo "c5 bench failed"; tail -20 $out/bench_c5.err; exit 1; }
  cat $out/bench_c5.json
fi
echo done
