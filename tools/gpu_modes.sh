#!/bin/bash
# join timing per strategy (direct / split / partitioned): tools/gpu_modes.sh TAG
tag=${1:-modes}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for mode in direct split partitioned; do
  timeout -k 10 200 python bench.py --only join --no-cpu --no-gather --join-mode $mode --join-steps 5 \
    > gpurun_out/${tag}_$mode.json 2> gpurun_out/${tag}_$mode.err || exit 1
  echo "$mode $(python -c "import json;d=json.load(open('gpurun_out/${tag}_$mode.json'))['pip_join'];print(round(d['ms_per_step'],2), d['matches'])")" >> gpurun_out/${tag}.txt
done
