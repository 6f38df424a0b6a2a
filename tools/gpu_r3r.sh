#!/bin/bash
# one box: a one-round relate A/B (product / coarse-core build / no core table), then the HEAD capture
set -e
tag=$1; cap=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/jq_variants.sh $tag 1 libgeomesa_hip l4_1024 nocore
bash tools/gpu_capture_r3.sh $cap
