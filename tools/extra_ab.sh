#!/bin/bash
# A/B of extra-leg kernels: GPU tests matching $TEST_K on $TEST_LIB, then bench --only extra per variant
# library, alternating 3 times, printing the legs named in KEYS.  usage: KEYS="z3_histogram ..." tools/extra_ab.sh TAG lib1 lib2 ...
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
( [ -n "$TEST_LIB" ] && export GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$TEST_LIB.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "${TEST_K:-stats}" --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 )
for i in 1 2 3; do
  for lib in "$@"; do
    GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so timeout -k 10 300 python bench.py --only extra --no-cpu --no-gather \
      --steps 10 > gpurun_out/${tag}_$lib.json 2> gpurun_out/${tag}_$lib.err
    python - "$tag" "$lib" "$i" $KEYS >> gpurun_out/${tag}_ab.txt <<'PY'
import json, sys
tag, lib, i = sys.argv[1:4]
x = json.load(open("gpurun_out/%s_%s.json" % (tag, lib)))["extra"]
print(lib, i, " ".join("%s %.4f" % (k, x[k]["ms_per_step"]) for k in sys.argv[4:]))
PY
  done
done
