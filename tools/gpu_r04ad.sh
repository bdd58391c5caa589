#!/bin/bash
# deep-pipelined 3x3 weight gradient (wgrad_h3d_kernel, DVIE_WG_DEEP)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04ad}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad.py > $out/pytest.log 2>&1 \
  || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for v in 1 0; do
  DVIE_WG_DEEP=$v timeout -k 10 200 python -u tools/wgrad_tune.py 10 '3x3 64->64|3x3 128->128|3x3 256->256' > $out/wg_deep_$v.txt 2>&1 || { tail $out/wg_deep_$v.txt; exit 1; }
  echo "deep=$v"; grep -v "^$" $out/wg_deep_$v.txt | tail -4
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py::test_inter_step_matches_reference \
  tests/test_gpu_configs.py::test_c2_bf16_step_256x512_b8_quality > $out/pytest2.log 2>&1 || { tail -30 $out/pytest2.log; exit 1; }
tail -1 $out/pytest2.log
bash tools/ab_env.sh DVIE_WG_DEEP 1 0 ${1:-r04ad}/ab_deep || exit 1
