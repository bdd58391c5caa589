#!/bin/bash
# conv_h8: early column barrier (default) vs the barrier after the last MFMAs; parity, micro, step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-h8b}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_epilogue.py::test_conv_h8_modes \
  > $out/pytest_h8.log 2>&1 || { tail -30 $out/pytest_h8.log; exit 1; }
tail -1 $out/pytest_h8.log
for e in 1 0 1 0; do
  DVIE_H8_EARLY=$e timeout -k 10 200 python -u tools/conv_tune.py -3 20 '128->128|256->256' > $out/tune_$e.txt 2>&1 || { tail $out/tune_$e.txt; exit 1; }
  echo "early=$e"; grep cfg $out/tune_$e.txt
done
bash tools/ab_env.sh DVIE_H8_EARLY 1 0 ${1:-h8b}/ab_early || exit 1
