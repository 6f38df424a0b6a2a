#!/bin/bash
# join + sort GPU tests, join A/B against a variant library, then the table leg (sort timing)
set -e
tag=${1:-run}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_join_faults.py tests/test_gpu_states.py tests/test_gpu_shortcuts.py tests/test_gpu_scan_join_ranges.py tests/test_gpu_arrow.py tests/test_gpu_index_build.py tests/test_gpu_dist.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
bash tools/jq_variants.sh ${tag} 2 "$@"
timeout -k 10 300 python -u bench.py --only z3,table --no-cpu > gpurun_out/${tag}_table.json 2> gpurun_out/${tag}_table.err
