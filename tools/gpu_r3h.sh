#!/bin/bash
# full GPU suite, then join variants A/B (alternating rounds on one box)
set -e
tag=${1:-run}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
bash tools/jq_variants.sh ${tag} 2 "$@"
