for c in 24576 32768; do
  timeout -k 10 300 python -u bench.py --only join --no-cpu --no-gather --steps 1 --warmup 0 --join-steps 3 --cells-per-poly $c > gpurun_out/r4h_dens_$c.json 2> gpurun_out/r4h_dens_$c.err || exit 1
  cp gpurun_out/bench_detail_n1.json gpurun_out/r4h_dens_$c.detail.json
done
