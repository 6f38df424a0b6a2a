#!/bin/bash
# A/B of Z3 key kernel variants (bench --only z3, 30 steps, alternating): tools/key_ab2.sh TAG lib1 lib2 ...
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  for lib in "$@"; do
    GEOMESA_HIP_LIB=$GRAFT_REPO_ROOT/geomesa_amd/lib/$lib.so timeout -k 10 200 python -u bench.py --only z3 --no-cpu --steps 30 \
      > gpurun_out/${tag}_k.json 2>/dev/null || exit 1
    echo "$lib $i $(python -c "import json;d=json.load(open('gpurun_out/${tag}_k.json'));print(round(d['ms_per_step'],4), d['roofline']['frac'])")" >> gpurun_out/${tag}_key.txt
  done
done
