#!/bin/bash
# filter-scan GPU tests on the default library (or $TEST_LIB), then the z3filter_scan leg of bench.py (--only extra),
# alternating the variant libraries 3 times.  usage: tools/filter_ab.sh TAG lib1 lib2 ...
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
( [ -n "$TEST_LIB" ] && export GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$TEST_LIB.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "filter or scan or query" --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 )
for i in 1 2 3; do
  for lib in "$@"; do
    GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so timeout -k 10 300 python bench.py --only extra --no-cpu --no-gather \
      --steps 10 > gpurun_out/${tag}_$lib.json 2> gpurun_out/${tag}_$lib.err
    python - "$tag" "$lib" "$i" >> gpurun_out/${tag}_ab.txt <<'PY'
import json, sys
tag, lib, i = sys.argv[1:]
x = json.load(open("gpurun_out/%s_%s.json" % (tag, lib)))["extra"]
e = x["z3filter_scan"]
print(lib, i, round(e["ms_per_step"], 4), e.get("roofline", {}).get("frac"),
      "query", round(x["query_scan"]["ms_per_step"], 4), "query_poly", round(x["query_scan_polygon"]["ms_per_step"], 4))
PY
  done
done
