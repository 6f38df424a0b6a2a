#!/bin/bash
# relate core rectangles: the row-predicate tests, then the join-leg A/B over block sizes and the no-core build
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_relate.py tests/test_gpu_shortcuts.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
bash tools/jq_variants.sh $tag 2 "$@"
