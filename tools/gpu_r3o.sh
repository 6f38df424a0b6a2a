#!/bin/bash
# histogram tests, then the histogram probe alternating product / variant
set -e
tag=$1; var=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stats.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python -u tools/hist_probe.py > gpurun_out/${tag}_prod_$r.txt 2>&1
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$var.so timeout -k 10 200 python -u tools/hist_probe.py > gpurun_out/${tag}_${var}_$r.txt 2>&1
done
