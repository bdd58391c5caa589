#!/bin/bash
# leak hunt: the C5 tests, then the CUDA memory left allocated and who holds it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-r04ag}; mkdir -p $out
timeout -k 10 900 python -u tools/mem_leak_probe.py --timeout 600 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_configs.py::test_c5_hrnet_1024x2048 > $out/leak.txt 2>&1 || { tail -40 $out/leak.txt; exit 1; }
tail -40 $out/leak.txt
