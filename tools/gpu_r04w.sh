#!/bin/bash
# r04: captured-step tests after the capture-keeps-one-stream change, then the round line:
# default bench + rocprof summary + C5 line with its per-op table, and the captured C2 step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-r04w}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_lanes.py \
  tests/test_gpu_dp.py tests/test_gpu_c5.py > $out/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/pytest.log | head; tail -20 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -1
bash tools/gpu_round.sh $tag skip-tests c5 > $out/round.log 2>&1 || { echo "round failed"; tail -30 $out/round.log; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['step_breakdown_ms'].get('weight_pack'))"
python3 -c "import json;d=json.load(open('$out/bench_c5.json'));print('c5', d['value'], d['ms_per_step'], d.get('attn'))"
timeout -k 10 300 python -u bench.py --graph 1 --no-cpu-baseline --profile-steps 0 > $out/c2_graph.json 2> $out/c2_graph.err || { tail -20 $out/c2_graph.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/c2_graph.json'));print('c2 captured', d['value'], d['ms_per_step'], d['eager_ms_per_step'])"
