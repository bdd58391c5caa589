mkdir -p gpurun_out/r03x
timeout -k 10 120 python -u tools/concur_micro.py 20 > gpurun_out/r03x/concur_fwd.txt 2>&1 || exit 1
timeout -k 10 180 python -u tools/concur_micro.py 10 bwd > gpurun_out/r03x/concur_bwd.txt 2>&1 || exit 1
cat gpurun_out/r03x/concur_*.txt
for c in 116 101 100 118; do
  DVIE_CONV1X1_WIDE=$c timeout -k 10 120 python -u tools/conv_epi_micro.py 8 256 512 64 256 1 30 > gpurun_out/r03x/epi_64_256_cfg$c.txt 2>&1 || exit 1
  echo "cfg $c"; grep -v amdgpu.ids gpurun_out/r03x/epi_64_256_cfg$c.txt
done
bash tools/ab_env.sh DVIE_CONV_NARROW 0 1 ab_narrow || exit 1
timeout -k 10 420 python -u bench.py --workload c5 --steps 5 --warmup 2 --ops-out gpurun_out/r03x/ops_c5.txt > gpurun_out/r03x/bench_c5.json 2> gpurun_out/r03x/bench_c5.err || exit 1
cat gpurun_out/r03x/bench_c5.json
