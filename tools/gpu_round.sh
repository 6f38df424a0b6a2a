#!/bin/bash
# One GPU call: parity tests, the default bench line, and a rocprofv3 kernel-stats run of the bench.
# usage (from the repo root on the GPU box): tools/gpu_round.sh TAG
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --steps 10 --join-steps 3 --no-cpu > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
