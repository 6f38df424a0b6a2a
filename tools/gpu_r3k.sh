#!/bin/bash
# sort tests, then the table leg under rocprofv3 kernel stats
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_dist.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python3 bench.py --only z3,table --no-cpu --steps 2 --warmup 1 > gpurun_out/${tag}.json 2> gpurun_out/${tag}.err
