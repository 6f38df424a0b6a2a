#!/bin/bash
# PMC passes (one group per rocprofv3 run, kernel trace only) over one bench leg.
# usage: tools/gpu_pmc_r3.sh TAG LEG   (LEG: join | table);  groups: PMC_GROUPS="A B;C D" or the default below
set -e
tag=$1; leg=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${tag}_pmc_${leg}; mkdir -p $out
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM"
  "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
)
if [ -n "$PMC_GROUPS" ]; then IFS=";" read -ra groups <<< "$PMC_GROUPS"; fi
cmd="python3 bench.py"
if [ "$leg" = join ]; then args="--only join --no-cpu --no-gather --steps 1 --warmup 0 --join-steps 1"
elif [ "$leg" = ranges ]; then cmd="python3 tools/ranges_probe.py"; args="100000"
elif [ "$leg" = hist ]; then cmd="python3 tools/hist_probe.py"; args=""
else args="--only z3,table --no-cpu --steps 1 --warmup 0"; fi
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $g -d $out/p$i -o run -- \
    $cmd $args > $out/p$i.log 2>&1 || { echo "pass $i ($g) failed: $?" >> $out/failed.txt; break; }
  i=$((i+1))
done
if [ "$leg" = join ]; then
  python3 tools/pmc_summary.py $out "k_pip_join_q<true" > $out/join.txt
  python3 tools/pmc_summary.py $out "k_pip_relate" > $out/relate.txt
elif [ "$leg" = hist ]; then
  python3 tools/pmc_summary.py $out "k_z3_hist_lds<1, false, true, false>" > $out/hist.txt
elif [ "$leg" = ranges ]; then
  python3 tools/pmc_summary.py $out "k_xzranges<3>" > $out/xz3.txt
  python3 tools/pmc_summary.py $out "k_xzranges<2>" > $out/xz2.txt
else
  python3 tools/pmc_summary.py $out "k_sort_scatter" > $out/scatter.txt
  python3 tools/pmc_summary.py $out "k_sort_hist" > $out/hist.txt
fi
