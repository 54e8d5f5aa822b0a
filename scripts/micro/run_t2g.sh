#!/bin/bash
# 4 x 4 lane-grid solver micro (t2g_check): timing and accuracy vs the
# row-per-lane solver and the 8 x 8 grid at D = 19 (and 11, 15).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/t2d
TAG=${TAG:-t2g}
for spec in "5 19 1 0" "5 19 4 3" "5 20 1 7" "4 15 1 0" "4 16 2 5"; do
  set -- $spec
  b=scripts/micro/bin/t2g_check$1
  [ -x $b ] || continue
  timeout -k 10 120 $b $2 16416 $3 $4 || exit 1
done 2>&1 | tee gpurun_out/t2d/${TAG}.log || exit 1
