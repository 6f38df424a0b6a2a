#!/bin/bash
# Collect PMC counters in separate rocprofv3 passes (one --pmc group per run, kernel-trace only).
# usage: tools/pmc_passes.sh OUTDIR -- python3 bench.py ...
set -e
out=$1; shift; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$out"
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
  "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_SMEM"
  "SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
)
# PMC_GROUPS="A B;C D" overrides the default passes
if [ -n "$PMC_GROUPS" ]; then IFS=";" read -ra groups <<< "$PMC_GROUPS"; fi
i=0
for g in "${groups[@]}"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc $g -d "$out/p$i" -o run -- "$@" > "$out/p$i.log" 2>&1
  i=$((i+1))
done
