# join grid density sweep on one box (bench join leg: the join and the row predicate), densities from
# $DENS (default "16384 20480"), two alternating rounds
i=0
for r in 1 2; do
  for c in ${DENS:-16384 20480}; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --only join --no-cpu --no-gather --steps 1 --warmup 0 --join-steps 3 --cells-per-poly $c > gpurun_out/${DTAG:-dens}_${c}_$i.json 2> gpurun_out/${DTAG:-dens}_${c}_$i.err || exit 1
    cp gpurun_out/bench_detail_n1.json gpurun_out/${DTAG:-dens}_${c}_$i.detail.json
  done
done
