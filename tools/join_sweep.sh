#!/bin/bash
# join timing sweep over library variants and grid densities (direct mode, no CPU baseline)
# usage: tools/join_sweep.sh TAG "lib1 lib2 ..." "cells1 cells2 ..."
tag=$1; libs=$2; cells=$3
for lib in $libs; do
  for c in $cells; do
    GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib timeout -k 10 200 python bench.py --only join --no-cpu --join-mode direct \
      --join-steps 3 --cells-per-poly $c > gpurun_out/${tag}_${lib%.so}_$c.json 2> gpurun_out/${tag}_${lib%.so}_$c.err || exit 1
  done
done
