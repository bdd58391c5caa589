#!/bin/bash
# Bench line + a rocprofv3 kernel TRACE (per-dispatch start/end, stream / queue ids) of the eager
# bench step with its executor lanes on, for the step timeline (tools/timeline.py).
# usage (via gpurun): bash tools/gpu_trace.sh <tag> [pytest args...]
set -o pipefail
tag=${1:-trace}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 600 --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/pytest.log | tail -30; exit 1; }
  tail -2 $out/pytest.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o t -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --profile-steps 0 --graph 0 > $out/trace.json 2> $out/trace.err || { echo "trace failed"; tail -20 $out/trace.err; exit 1; }
find $out/trace -name '*kernel_trace.csv' | head -2
echo done
