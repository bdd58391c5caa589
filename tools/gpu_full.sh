#!/bin/bash
# The whole GPU suite, smoke, the bench line and the rocprofv3 kernel-trace summary of the bench.
# usage (via gpurun): bash tools/gpu_full.sh TAG
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" $out/pytest_gpu.log | tail -30; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 420 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_breakdown_ms'])"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 --graph 0 > $out/bench_prof.json 2> $out/bench_prof.err || { echo "rocprof failed"; tail -20 $out/bench_prof.err; exit 1; }
find $out/prof -name '*kernel_trace.csv' -delete
echo done
