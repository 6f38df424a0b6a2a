#!/bin/bash
# join parity tests + grid-density / mode sweep (GPU box)
set -e
out=${1:-gpurun_out/sweep.log}
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "pip or contains or join" > gpurun_out/t.log 2>&1
for m in direct partitioned; do
  for c in 1024 2048 4096; do
    timeout -k 10 200 python bench.py --only join --no-cpu --cells-per-poly $c --join-mode $m --join-steps 5 >> "$out" 2>&1
  done
done
