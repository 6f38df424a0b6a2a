#!/bin/bash
# Round-end GPU capture, part B: rocprofv3 kernel stats of the bench, then one counter group per
# run (kernel trace only): FETCH_SIZE / WRITE_SIZE of the streaming legs, the table sort and the
# join, and the join's FP64 VALU instruction count.  usage: tools/gpu_prof3.sh TAG
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --steps 10 --join-steps 3 --no-cpu > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
i=0
for g in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $g -d gpurun_out/${tag}_pmc/p$i -o run -- \
    python3 bench.py --only z3,extra,table --no-cpu --steps 2 --warmup 1 > gpurun_out/${tag}_pmc$i.log 2>&1
  i=$((i+1))
done
for g in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU_FLOPS_FP64; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $g -d gpurun_out/${tag}_pmc/p$i -o run -- \
    python3 bench.py --only join --no-cpu --steps 1 --warmup 0 --join-steps 1 --join-mode direct \
    > gpurun_out/${tag}_pmc$i.log 2>&1
  i=$((i+1))
done
