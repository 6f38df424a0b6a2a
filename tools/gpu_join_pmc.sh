#!/bin/bash
# Join-kernel counters, one --pmc group per rocprofv3 run (kernel trace only):
# occupancy / wait, instruction mix, L2 hit / miss, HBM bytes.  usage: tools/gpu_join_pmc.sh TAG
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/${tag}_jpmc
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP64"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"
)
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $g -d gpurun_out/${tag}_jpmc/p$i -o run -- \
    python3 bench.py --only join --no-cpu --no-gather --steps 1 --warmup 0 --join-steps 1 \
    > gpurun_out/${tag}_jpmc/p$i.log 2>&1
  i=$((i+1))
done
python3 tools/pmc_summary.py gpurun_out/${tag}_jpmc "k_pip_join_q<true" > gpurun_out/${tag}_jpmc/join.txt
python3 tools/pmc_summary.py gpurun_out/${tag}_jpmc "k_pip_relate" > gpurun_out/${tag}_jpmc/relate.txt
