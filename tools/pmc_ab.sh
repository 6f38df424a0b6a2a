#!/bin/bash
# PMC A/B of the join kernel across library variants on one box.
# usage: tools/pmc_ab.sh TAG "variant ..."   (variant "main" = the default build)
tag=$1
export PMC_GROUPS="${PMC_GROUPS-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VALU_FLOPS_FP64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM}"
for name in $2; do
  v=""; [ "$name" != main ] && v="_$name"
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/libgeomesa_hip$v.so tools/pmc_passes.sh gpurun_out/pmc_${tag}_$name -- python3 bench.py --only join --no-cpu --no-gather --join-steps 2 --join-mode direct || exit 1
  echo "== $name" >> gpurun_out/pmc_${tag}.txt
  python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_$name "k_pip_join<true, false, false" >> gpurun_out/pmc_${tag}.txt
done
cat gpurun_out/pmc_${tag}.txt
