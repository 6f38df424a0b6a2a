#!/bin/bash
# unroll A/B of the curve kernels: bench --only z3,extra per variant library, alternating 2 times;
# then the curve GPU tests on each variant.  usage: tools/curve_ab.sh TAG lib1 lib2 ...
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so timeout -k 10 300 python bench.py --only z3,extra --no-cpu --no-gather \
      --steps 10 > gpurun_out/${tag}_$lib.json 2> gpurun_out/${tag}_$lib.err
    python - "$tag" "$lib" "$i" >> gpurun_out/${tag}_ab.txt <<'PY'
import json, sys
tag, lib, i = sys.argv[1:]
d = json.load(open("gpurun_out/%s_%s.json" % (tag, lib)))
x = d["extra"]
print(lib, i, "key", round(d["ms_per_step"], 3), " ".join("%s %.3f" % (k, x[k]["ms_per_step"]) for k in
      ("z3_invert", "z2_index", "z2_invert", "arrow_z3_keys", "xz2_index", "xz3_index")))
PY
  done
done
for lib in "$@"; do
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
    -k "curve or z3 or z2 or xz or key or arrow" --timeout 120 --timeout-method thread > gpurun_out/${tag}_${lib}_tests.log 2>&1
  echo "$lib $(tail -1 gpurun_out/${tag}_${lib}_tests.log)" >> gpurun_out/${tag}_ab.txt
done
