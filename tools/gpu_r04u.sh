#!/bin/bash
# r04: attention on the matrix cores -- parity, then the C5 line with it on / off (same box),
# then the default bench line with its rocprof kernel summary
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04u}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_refine.py tests/test_gpu_c5.py > $out/pytest.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/pytest.log | head; tail -20 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -2
for v in 1 0; do
  DVIE_ATTN_MFMA=$v timeout -k 10 500 python -u bench.py --workload c5 --no-cpu-baseline --ops-out $out/ops_c5_$v.txt > $out/c5_$v.json 2> $out/c5_$v.err || { echo "c5 bench failed"; tail -20 $out/c5_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/c5_$v.json'));print('attn_mfma=$v', d['value'], d['ms_per_step'], d.get('attn'))"
done
