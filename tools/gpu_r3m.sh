#!/bin/bash
# ranges tests against variant libraries, then the probe alternating product / variants
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_scan_join_ranges.py tests/test_gpu_boundary.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests_$v.log 2>&1
done
for r in 1 2; do
  timeout -k 10 200 python -u tools/ranges_probe.py 100000 > gpurun_out/${tag}_prod_$r.txt 2>&1
  for v in "$@"; do
    GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$v.so timeout -k 10 200 python -u tools/ranges_probe.py 100000 > gpurun_out/${tag}_${v}_$r.txt 2>&1
  done
done
