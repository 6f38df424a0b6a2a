#!/bin/bash
# A/B of join library variants on one box, alternating rounds: tools/jq_variants.sh TAG ROUNDS lib1 lib2 ...
# (libN = geomesa_amd/lib/<libN>.so; "legacy" = the product library with GM_PIP_JOIN_LEGACY=1)
set -e
tag=$1; rounds=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    # "legacy" = the product library's round-2 kernel; "legacy:<lib>" = that kernel in variant <lib>
    unset GM_PIP_JOIN_LEGACY GM_PIP_RELATE_SCALAR GM_PIP_NO_CORE; env_lib=""
    case "$lib" in
      scalar) export GM_PIP_RELATE_SCALAR=1 ;;   # the product library, row-by-row relate loads
      nocore) export GM_PIP_NO_CORE=1 ;;         # the product library, no core rectangles
      legacy) export GM_PIP_JOIN_LEGACY=1 ;;
      legacy:*) export GM_PIP_JOIN_LEGACY=1; env_lib="GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/${lib#legacy:}.so" ;;
      *) env_lib="GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib.so" ;;
    esac
    env $env_lib timeout -k 10 300 python bench.py --only join --no-cpu --no-gather --join-steps 5 \
      > gpurun_out/${tag}_${lib//:/_}_$r.json 2> gpurun_out/${tag}_${lib//:/_}_$r.err
    python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_${lib//:/_}_$r.json').read().strip().splitlines()[-1])['pip_join']; print('$lib', $r, round(d['ms_per_step'],3), d['matches'], d.get('row_predicate_ms'))" >> gpurun_out/${tag}_ab.txt
  done
done
unset GM_PIP_JOIN_LEGACY GM_PIP_RELATE_SCALAR GM_PIP_NO_CORE
