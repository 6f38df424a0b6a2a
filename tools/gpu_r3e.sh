#!/bin/bash
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
bash tools/jq_variants.sh ${tag} 2 libgeomesa_hip legacy
