#!/bin/bash
# Full GPU round: parity tests, bench line, rocprof kernel stats, and FETCH/WRITE PMC passes of the
# streaming kernels (z3 + extra legs).  usage: tools/gpu_round2.sh TAG
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --steps 10 --join-steps 3 --no-cpu > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d gpurun_out/${tag}_pmc/p0 -o run -- \
  python3 bench.py --only z3,extra --no-cpu --steps 2 --warmup 1 > gpurun_out/${tag}_pmc0.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d gpurun_out/${tag}_pmc/p1 -o run -- \
  python3 bench.py --only z3,extra --no-cpu --steps 2 --warmup 1 > gpurun_out/${tag}_pmc1.log 2>&1
