#!/bin/bash
# timing experiments on variant builds of the join (GM_JX_* macros; results of those builds are not
# correct joins, only timings).  usage: tools/join_experiments.sh TAG "lib..." "opts;opts;..."
tag=$1; libs=$2; IFS=";" read -ra opts <<< "$3"
for lib in $libs; do
 for opt in "${opts[@]}"; do
  GEOMESA_HIP_LIB=$PWD/geomesa_amd/lib/$lib timeout -k 10 200 python bench.py --only join --no-cpu --join-steps 3 $opt > gpurun_out/jx.tmp 2>&1 || exit 1
  echo "$lib [$opt] $(python -c "import json;d=json.loads(open('gpurun_out/jx.tmp').read().strip().split(chr(10))[-1]);print(round(d['pip_join']['ms_per_step'],2), d['pip_join']['matches'])")" >> gpurun_out/${tag}_jx.txt
 done
done
