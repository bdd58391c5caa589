#!/bin/bash
# r04: GPU tests touched by this round's changes, then a bench line with its per-op table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04a}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_gpu_head3.py \
  tests/test_gpu_gan.py tests/test_gpu_vae.py tests/test_gpu_refine.py tests/test_gpu_c5.py::test_extra_stage3_step_matches_oracle \
  tests/test_gpu_train.py tests/test_gpu_lanes.py tests/test_gpu_parity.py::test_warp_multi_tile tests/test_gpu_parity.py::test_warp tests/test_gpu_graph.py "tests/test_gpu_configs.py::test_c4_intergan_step_512x1024" \
  tests/test_gpu_metrics.py > $out/pytest.log 2>&1
rc=$?; grep -E "passed|failed|gradients vs|Error|assert|worst" $out/pytest.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --ops-out $out/ops.txt > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['step_breakdown_ms'])"
head -20 $out/ops.txt
