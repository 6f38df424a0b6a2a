#!/bin/bash
# A/B of the Z3 key kernel on one box: register spreads (default lib) vs the LDS spread table
# (build it first: python -m geomesa_amd.build -DGM_KEY_TABLE --out=geomesa_amd/lib/libgeomesa_hip_tab.so).
# Round 1: 5.88 / 5.83 ms (registers) vs 6.02 / 5.81 ms (table) -- within noise, registers kept.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --only z3 --no-cpu --steps 30 > gpurun_out/ab_reg_$i.json 2>/dev/null
  GEOMESA_HIP_LIB=$GRAFT_REPO_ROOT/geomesa_amd/lib/libgeomesa_hip_tab.so timeout -k 10 200 python -u bench.py --only z3 --no-cpu --steps 30 > gpurun_out/ab_tab_$i.json 2>/dev/null
done
