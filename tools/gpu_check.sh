#!/bin/bash
# Selected GPU tests (-s output kept), then the bench line with its per-op table.
# usage (via gpurun): bash tools/gpu_check.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest "$@" -x -v -s --timeout 600 --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert|rel L2" $out/pytest.log | tail -30; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --ops-out $out/ops.txt > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_breakdown_ms'])"
