#!/bin/bash
# ranges tests, then the ranges probe: product library vs a variant (alternating)
set -e
tag=${1:-run}; var=${2:-rold}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_join_ranges.py tests/test_gpu_boundary.py tests/test_gpu_legacy.py tests/test_gpu_partitions.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python -u tools/ranges_probe.py 100000 > gpurun_out/${tag}_prod_$r.txt 2>&1
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$var.so timeout -k 10 200 python -u tools/ranges_probe.py 100000 > gpurun_out/${tag}_${var}_$r.txt 2>&1
done
