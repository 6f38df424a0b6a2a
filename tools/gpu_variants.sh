#!/bin/bash
# parity tests on the default build, then the join bench for each variant library
set -e
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "pip or contains or join" > gpurun_out/t.log 2>&1
for lib in geomesa_amd/lib/libgeomesa_hip*.so; do
  for c in 2048 4096; do
    echo "LIB $lib" >> gpurun_out/var.log
    GEOMESA_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --only join --no-cpu --cells-per-poly $c --join-mode direct --join-steps 5 >> gpurun_out/var.log 2>&1
  done
done
