#!/bin/bash
# 2D solver micro: phase timings of each build in scripts/micro/bin and a
# bit-identity check of its filters against the HEAD build (t2d_head<NB>).
# usage: VARIANTS="pack" bash scripts/micro/run_t2d.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/t2d
TAG=${TAG:-t2d}
for v in head ${VARIANTS:-pack}; do
  for spec in "5 39 1 0" "5 39 4 3" "3 19 1 0"; do
    set -- $spec
    b=scripts/micro/bin/t2d_$v$1
    [ -x $b ] || continue
    echo "== $v NB=$1 D=$2 R=$3 ref=$4"
    timeout -k 10 120 $b $2 16416 $3 $4 gpurun_out/t2d/w_${v}_$1_$2_$3.bin || exit 1
    if [ "$v" != head ]; then
      cmp -s gpurun_out/t2d/w_head_$1_$2_$3.bin gpurun_out/t2d/w_${v}_$1_$2_$3.bin && echo "  bit-identical to head" || echo "  DIFFERS from head"
    fi
  done
done 2>&1 | tee gpurun_out/t2d/${TAG}.log || exit 1
# SQ counters per phase kernel (phase2d<0..5>) of the last variant
if [ -n "$PMC" ]; then
  v=${PMC}
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY \
    --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/t2d/pmc_$v -o pmc -- $GRAFT_REPO_ROOT/scripts/micro/bin/t2d_${v}5 39 16416 1 0 > $GRAFT_REPO_ROOT/gpurun_out/t2d/pmc_$v.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT
fi
