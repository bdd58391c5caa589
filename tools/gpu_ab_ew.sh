#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06l
timeout -k 10 300 python -u -m pytest tests/test_gpu_ew.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06l/pytest.log 2>&1 || { tail -30 gpurun_out/r06l/pytest.log; exit 1; }
tail -1 gpurun_out/r06l/pytest.log
bash tools/ab_env_ops.sh r06l - DVIE_EW_UPT22=0 "DVIE_EW_FUSER=0 DVIE_EW_UPT22=0" - DVIE_EW_UPT22=0 "DVIE_EW_FUSER=0 DVIE_EW_UPT22=0"
