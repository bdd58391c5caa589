# Does the hipGraph executor run the captured side-stream lanes concurrently?  Same box:
# graph replay (default), graph replay with DEBUG_HIP_FORCE_GRAPH_QUEUES, eager replay; lanes on.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03q; mkdir -p $out
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0 $BARGS > $out/$tag.json 2> $out/$tag.err || { tail -5 $out/$tag.err; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' $out/$tag.json)"
}
for r in 1 2; do
  BARGS="" run graph_lanes0_$r DVIE_OP_LANES=0
  BARGS="" run graph_lanes1_$r DVIE_OP_LANES=1
  BARGS="" run graph_q4_lanes1_$r DVIE_OP_LANES=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
  BARGS="" run graph_q2_lanes1_$r DVIE_OP_LANES=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
  BARGS="--graph 0" run eager_lanes1_$r DVIE_OP_LANES=1
done
