#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
pkg=deep_video_interpolation_extrapolation_amd/libdvie.so
mkdir -p gpurun_out/skipchk; cp $pkg gpurun_out/skipchk/orig.so
trap 'cp gpurun_out/skipchk/orig.so $pkg' EXIT
timeout -k 10 120 python -u tools/skip_check.py 2>&1 | grep skip
cp tools/probe/libdvie_tdbg.so $pkg || exit 1
for m in 0 28; do DVIE_SKIP_KINDS=$m timeout -k 10 120 python -u tools/skip_check.py 2>&1 | grep skip; done
