#!/bin/bash
# 3x3 weight gradient with the fragment pipeline (DVIE_WG_PIPE) + warp XCD bands
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04ab}; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad.py tests/test_gpu_parity.py > $out/pytest.log 2>&1 \
  || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for v in 1 0; do
  DVIE_WG_PIPE=$v timeout -k 10 200 python -u tools/wgrad_tune.py 10 '3x3 64->64|3x3 128->128|3x3 256->256' > $out/wg_pipe_$v.txt 2>&1 || { tail $out/wg_pipe_$v.txt; exit 1; }
  echo "pipe=$v"; grep -v "^$" $out/wg_pipe_$v.txt | tail -4
done
timeout -k 10 300 python -u tools/warp_ab.py DVIE_WARP_XCD 1 0 3 > $out/warp_xcd.txt 2>&1 || { tail -20 $out/warp_xcd.txt; exit 1; }
cat $out/warp_xcd.txt
bash tools/ab_env.sh DVIE_WG_PIPE 1 0 ${1:-r04ab}/ab_pipe || exit 1
