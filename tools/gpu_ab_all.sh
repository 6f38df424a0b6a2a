#!/bin/bash
# full -m gpu suite on the default library, then the join / relate / query legs of bench.py for
# each variant library.  usage: tools/gpu_ab_all.sh TAG lib1 lib2 ...
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
for lib in "$@"; do
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so timeout -k 10 300 python bench.py --only join,extra --no-cpu --no-gather \
    --join-steps 5 --steps 4 > gpurun_out/${tag}_$lib.json 2> gpurun_out/${tag}_$lib.err
  python - "$tag" "$lib" >> gpurun_out/${tag}_ab.txt <<'PY'
import json, sys
tag, lib = sys.argv[1:]
d = json.load(open("gpurun_out/%s_%s.json" % (tag, lib)))
j, e = d["pip_join"], d["extra"]
print(lib, "join", round(j["ms_per_step"], 2), j["matches"], "relate", round(j["row_predicate"]["ms_per_step"], 2),
      "query", round(e["query_scan"]["ms_per_step"], 3), "query_poly", round(e["query_scan_polygon"]["ms_per_step"], 3),
      e["query_scan_polygon"].get("matches"))
PY
done
