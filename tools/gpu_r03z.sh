# lanes under eager replay vs hipGraph replay (does the graph keep the side streams' concurrency?)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03z; mkdir -p $out
run() {  # tag env... -- bench args
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0 $BARGS > $out/$tag.json 2> $out/$tag.err || { tail -5 $out/$tag.err; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $out/$tag.json)"
}
for r in 1 2; do
  BARGS="--graph 0" run eager_lanes0_$r DVIE_OP_LANES=0
  BARGS="--graph 0" run eager_lanes1_$r DVIE_OP_LANES=1
  BARGS="" run graph_nopc_lanes0_$r DVIE_OP_LANES=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  BARGS="" run graph_nopc_lanes1_$r DVIE_OP_LANES=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" $out/pytest.log | head -20; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
