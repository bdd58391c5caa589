#!/bin/bash
# r04: the eight-row halo conv's parity cases first, then the GPU tests touched by this round,
# then bench lines with the eight-row kernel on and off (same box) and the per-op table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04c}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_epilogue.py::test_conv_h8_modes \
  > $out/pytest_h8.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" $out/pytest_h8.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_gpu_train.py tests/test_gpu_lanes.py \
  tests/test_gpu_parity.py::test_warp_multi_tile tests/test_gpu_parity.py::test_warp tests/test_gpu_graph.py \
  tests/test_gpu_configs.py::test_c2_bf16_step_256x512_b8_quality tests/test_gpu_configs.py::test_c3_extra_step_256x512 \
  "tests/test_gpu_configs.py::test_c4_intergan_step_512x1024" tests/test_gpu_metrics.py tests/test_gpu_conv_epilogue.py > $out/pytest.log 2>&1
rc=$?; grep -E "passed|failed|gradients vs|Error|assert|worst" $out/pytest.log | tail -60
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  DVIE_CONV_H8=$v timeout -k 10 420 python -u bench.py --no-cpu-baseline --profile-steps 0 > $out/ab_h8_$v.json 2>> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$out/ab_h8_$v.json'));print('h8=$v',d['value'],d['ms_per_step'])"
done
timeout -k 10 420 python -u bench.py --ops-out $out/ops.txt > $out/bench.json 2>> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['step_breakdown_ms'])"
head -30 $out/ops.txt
