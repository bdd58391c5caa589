#!/bin/bash
# r04: pipelined attention kernels, frozen-VGG pack skipped after the first forward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04z}; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_refine.py tests/test_gpu_train.py \
  tests/test_gpu_metrics.py tests/test_gpu_configs.py::test_c2_bf16_step_256x512_b8_quality tests/test_gpu_graph.py > $out/pytest.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/pytest.log | head; tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 420 python -u bench.py --no-cpu-baseline --ops-out $out/ops.txt > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print('c2', d['value'], d['ms_per_step'], d['step_breakdown_ms'])"
timeout -k 10 500 python -u bench.py --workload c5 --no-cpu-baseline --ops-out $out/ops_c5.txt > $out/c5.json 2> $out/c5.err || { tail -20 $out/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/c5.json'));print('c5', d['value'], d['ms_per_step'], d.get('attn'), d['step_breakdown_ms'].get('weight_pack'))"
