#!/bin/bash
# relate / join tests against variant libraries, then join + row-predicate A/B (alternating)
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_relate.py tests/test_gpu_shortcuts.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests_$v.log 2>&1
done
bash tools/jq_variants.sh ${tag} 2 libgeomesa_hip "$@"
