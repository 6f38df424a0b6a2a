#!/bin/bash
# join strategy check: parity tests of the join paths, then partitioned vs direct timings and a
# rocprofv3 kernel summary of the partitioned pass.  usage: tools/gpu_join_tri.sh TAG [pytest -k expr]
set -e
tag=${1:-tri}; kexpr=${2:-"join or states or partition"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$kexpr" \
  > gpurun_out/${tag}_tests.log 2>&1
for mode in partitioned direct; do
  timeout -k 10 200 python -u bench.py --only join --no-cpu --no-gather --join-mode $mode --join-steps 5 \
    > gpurun_out/${tag}_$mode.json 2> gpurun_out/${tag}_$mode.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --only join --no-cpu --no-gather --join-mode partitioned --join-steps 3 > gpurun_out/${tag}_prof.json 2> gpurun_out/${tag}_prof.err
