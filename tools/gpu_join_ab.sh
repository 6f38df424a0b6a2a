#!/bin/bash
# join parity tests on the default library, then A/B timings of variant libraries.
# usage: tools/gpu_join_ab.sh TAG lib1 lib2 ...
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "join or states or partition or relate or query" > gpurun_out/${tag}_tests.log 2>&1
bash tools/jx_run.sh $tag "$@"
