#!/bin/bash
# sort parity + timing, join kernel stats and PMC
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_sorttests.log 2>&1
timeout -k 10 300 python -u bench.py --only table --no-cpu > gpurun_out/${tag}_table.json 2> gpurun_out/${tag}_table.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --only join --no-cpu --no-gather --steps 1 --warmup 0 --join-steps 3 > gpurun_out/${tag}_prof_join.json 2> gpurun_out/${tag}_prof_join.err
bash tools/gpu_join_pmc.sh ${tag}
