#!/bin/bash
# one box: the relate A/B (tools/gpu_r3p.sh) and then the ranges probe alternating product / RVAR
set -e
tag=$1; rvar=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_r3p.sh $tag "$@"
for r in 1 2; do
  timeout -k 10 200 python -u tools/ranges_probe.py > gpurun_out/${tag}_rprod_$r.txt 2>&1
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$rvar.so timeout -k 10 200 python -u tools/ranges_probe.py > gpurun_out/${tag}_r${rvar}_$r.txt 2>&1
done
