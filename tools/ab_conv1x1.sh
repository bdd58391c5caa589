set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for r in 1 2; do
 for w in 102 116; do
  DVIE_CONV1X1_WIDE=$w timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0 > gpurun_out/ab/b_${w}_$r.json 2>/dev/null || exit 1
  echo "$w $r $(grep -o '"value": [0-9.]*' gpurun_out/ab/b_${w}_$r.json)"
 done
done
