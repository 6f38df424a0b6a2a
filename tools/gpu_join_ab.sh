#!/bin/bash
# A/B of the staged direct join (k_pip_join_q) against the round-2 kernel (GM_PIP_JOIN_LEGACY=1) on
# one box, alternating, plus the join parity tests.  usage: tools/gpu_join_ab.sh TAG [tests]
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$2" != "notests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_join_faults.py tests/test_gpu_scan_join_ranges.py tests/test_gpu_states.py \
    tests/test_gpu_shortcuts.py tests/test_gpu_arrow.py tests/test_gpu_relate.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_jtests.log 2>&1
fi
for r in 1 2; do
  for v in new legacy; do
    if [ $v = legacy ]; then export GM_PIP_JOIN_LEGACY=1; else unset GM_PIP_JOIN_LEGACY; fi
    timeout -k 10 300 python -u bench.py --only join --no-cpu --no-gather --join-steps 5 \
      > gpurun_out/${tag}_${v}_$r.json 2> gpurun_out/${tag}_${v}_$r.err
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_${v}_$r.json').read().strip().splitlines()[-1])['pip_join']; print('$v', $r, round(d['ms_per_step'],3), d['matches'])" >> gpurun_out/${tag}_ab.txt
  done
done
unset GM_PIP_JOIN_LEGACY
