#!/bin/bash
# sort timing per library variant: tools/gpu_sort_ab.sh TAG lib1 lib2 ...
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    echo "$lib $i $(GM_SORT_PROBE_NOCHECK=1 GEOMESA_HIP_LIB=$GRAFT_REPO_ROOT/geomesa_amd/lib/$lib.so timeout -k 10 200 python tools/sort_probe.py 2>&1 | tail -1)" >> gpurun_out/${tag}_sort.txt || exit 1
  done
done
