#!/bin/bash
# Round-3 GPU capture: smoke, the full -m gpu suite, the default bench line, gather-policy probe.
# usage: tools/gpu_r3a.sh TAG
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
if [ -x tools/gather_probe2 ]; then timeout -k 10 120 tools/gather_probe2 > gpurun_out/${tag}_gather2.log 2>&1; fi
if [ -n "$WITH_PMC" ]; then bash tools/gpu_join_pmc.sh ${tag}; fi
