#!/bin/bash
# r04: the LDS-tiled weight pack -- every plan family's parity tests, then the bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04y}; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py \
  tests/test_gpu_vae.py tests/test_gpu_gan.py tests/test_gpu_unet.py tests/test_gpu_extra.py \
  tests/test_gpu_configs.py::test_c2_bf16_step_256x512_b8_quality tests/test_gpu_head3.py > $out/pytest.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/pytest.log | head; tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 420 python -u bench.py --no-cpu-baseline --ops-out $out/ops.txt > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print('c2', d['value'], d['ms_per_step'], d['step_breakdown_ms'])"
