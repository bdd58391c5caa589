#!/bin/bash
# strip conv with the B-fragment pipeline (DVIE_CONV_STRIP=4) vs mode 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04ac}; mkdir -p $out
DVIE_CONV_STRIP=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_conv_epilogue.py -k "conv" > $out/pytest.log 2>&1 \
  || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for v in 4 2; do
  DVIE_CONV_STRIP=$v timeout -k 10 200 python -u tools/conv_tune.py -3 20 '3x3 64->64|3x3 32->32' > $out/strip_$v.txt 2>&1 || { tail $out/strip_$v.txt; exit 1; }
  echo "strip=$v"; grep -v "^$" $out/strip_$v.txt | tail -6
done
bash tools/ab_env.sh DVIE_CONV_STRIP 4 2 ${1:-r04ac}/ab_strip || exit 1
