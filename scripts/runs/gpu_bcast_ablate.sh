#!/bin/bash
# Diagnostic: broadcast-kernel time under ablation masks (DANSE_BCAST_ABLATE:
# 1 = skip analyses, 2 = skip z synthesis/analysis, 4 = skip estimate
# synthesis).  Results are wrong under ablation; only the kernel time matters.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for M in ${MASKS:-0 1 2 4 7}; do
  DANSE_BCAST_ABLATE=$M timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abl_$M -o kt --output-format csv -- python bench.py --steps 1 --warmup 1 --scenes ${S:-31} --no-cpu-baseline > gpurun_out/abl_$M.log 2>&1 || { echo "mask $M failed"; tail -5 gpurun_out/abl_$M.log; exit 1; }
  echo "mask $M: $(grep bcast_kernel gpurun_out/abl_$M/kt_kernel_stats.csv | cut -d, -f2-4)"
done
