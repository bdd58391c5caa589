#!/bin/bash
# One GPU-box pass for BASELINE config 5: its tests, then the c5 bench line with a per-op table.
# usage (from the repo root, via gpurun): bash tools/gpu_c5.sh <tag> [pytest selection...]
set -o pipefail
tag=${1:-c5}
shift
sel=${@:-tests/test_gpu_c5.py}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 700 python -u -m pytest $sel -x -v -s --timeout 650 --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
grep -E "PASS|FAIL|C5|median" $out/pytest.log | tail -20
timeout -k 10 420 python -u bench.py --workload c5 --steps 5 --warmup 2 --ops-out $out/ops_c5.txt > $out/bench_c5.json 2> $out/bench_c5.err || { echo "bench failed"; tail -20 $out/bench_c5.err; exit 1; }
cat $out/bench_c5.json
head -40 $out/ops_c5.txt
echo done
