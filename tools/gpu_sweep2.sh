#!/bin/bash
# join density x coarse-factor sweep: tools/gpu_sweep2.sh TAG "libs" "cells"
tag=$1; libs=$2; cells=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in $libs; do
  for c in $cells; do
    GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so timeout -k 10 200 python bench.py --only join --no-cpu --no-gather \
      --join-steps 4 --cells-per-poly $c > gpurun_out/sw.json 2> gpurun_out/sw.err || exit 1
    echo "$lib $c $(python -c "import json;d=json.load(open('gpurun_out/sw.json'))['pip_join'];print(round(d['ms_per_step'],2), d['matches'], d['index_build_s'], d['index']['cells'])")" >> gpurun_out/${tag}_sweep.txt
  done
done
