#!/bin/bash
# Round-3 capture of one tree: full GPU suite, smoke, the default bench line, then rocprofv3 kernel
# stats + PMC traffic passes (tools/gpu_prof3.sh).  usage: tools/gpu_capture_r3.sh TAG
set -e
tag=${1:-cap}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
cp gpurun_out/bench_detail_n1.json gpurun_out/${tag}_bench_detail.json
bash tools/gpu_prof3.sh ${tag}
