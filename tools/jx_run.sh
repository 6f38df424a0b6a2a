#!/bin/bash
# time the join with each variant library: tools/jx_run.sh TAG lib1 lib2 ...
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so timeout -k 10 200 python bench.py --only join --no-cpu --no-gather --join-steps 5 \
    > gpurun_out/${tag}_$lib.json 2> gpurun_out/${tag}_$lib.err || exit 1
  echo "$lib $(python -c "import json;d=json.load(open('gpurun_out/${tag}_$lib.json'))['pip_join'];print(round(d['ms_per_step'],2), d['matches'], round(d['row_predicate']['ms_per_step'],2))")" >> gpurun_out/${tag}_jx.txt
done
