#!/bin/bash
# join-family GPU tests, then join variants A/B (alternating rounds on one box)
set -e
tag=${1:-run}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_faults.py tests/test_gpu_states.py tests/test_gpu_shortcuts.py tests/test_gpu_scan_join_ranges.py tests/test_gpu_arrow.py tests/test_gpu_index_build.py tests/test_gpu_dist.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
bash tools/jq_variants.sh ${tag} 2 "$@"
