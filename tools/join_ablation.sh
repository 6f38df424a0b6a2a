#!/bin/bash
# join timing per variant build (GM_JX_* macros: timing only, not correct joins) and per strategy
# usage: tools/join_ablation.sh TAG
tag=$1
out=gpurun_out/${tag}_ablation.txt
: > $out
for name in ${VARIANTS-main noblob nofine}; do
  v=""; [ "$name" != main ] && v="_$name"
  for mode in ${MODES-direct split}; do
    GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/libgeomesa_hip$v.so timeout -k 10 200 python bench.py --only join --no-cpu --no-gather --join-steps 5 --join-mode $mode > gpurun_out/jx.tmp 2>gpurun_out/jx.err || exit 1
    echo "lib$v $mode $(python -c "import json;d=json.loads(open('gpurun_out/jx.tmp').read().strip().split(chr(10))[-1]);p=d['pip_join'];print(round(p['ms_per_step'],2), p['matches'], round(p['row_predicate']['ms_per_step'],2))")" >> $out
  done
done
cat $out
