#!/bin/bash
# Round-3 closing evidence, part 2: the default bench line (B, B at S=1
# launch-per-round / grid / resident, N2; PMC traffic; CPU baselines), the
# config C line, rocprofv3 kernel statistics of B, N2, C and the resident
# run, and the resident kernel's HBM traffic counters.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3z}
timeout -k 10 600 python bench.py > gpurun_out/bench_full_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_full_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_full_$TAG.log | cut -c1-200
timeout -k 10 300 python bench.py --workload C --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_C_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_C_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_C_$TAG.log | cut -c1-200
for W in B N2 C; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof${W}_$TAG -o kt --output-format csv -- python bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/prof${W}_$TAG.log 2>&1 || { tail -20 gpurun_out/prof${W}_$TAG.log; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/profRes_$TAG -o kt --output-format csv -- python bench.py --workload B --scenes 1 --resident --no-extra --no-cpu-baseline --no-traffic --steps 2 --warmup 1 > gpurun_out/profRes_$TAG.log 2>&1 || { tail -20 gpurun_out/profRes_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcRes1_$TAG -o pmc --output-format csv -- python bench.py --workload B --scenes 1 --resident --no-extra --no-cpu-baseline --no-traffic --steps 1 --warmup 0 > gpurun_out/pmcRes1_$TAG.log 2>&1 || { tail -20 gpurun_out/pmcRes1_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcRes2_$TAG -o pmc --output-format csv -- python bench.py --workload B --scenes 1 --resident --no-extra --no-cpu-baseline --no-traffic --steps 1 --warmup 0 > gpurun_out/pmcRes2_$TAG.log 2>&1 || { tail -20 gpurun_out/pmcRes2_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmcRes3_$TAG -o pmc --output-format csv -- python bench.py --workload B --scenes 1 --resident --no-extra --no-cpu-baseline --no-traffic --steps 1 --warmup 0 > gpurun_out/pmcRes3_$TAG.log 2>&1 || { tail -20 gpurun_out/pmcRes3_$TAG.log; exit 1; }
ls gpurun_out/pmcRes1_$TAG gpurun_out/pmcRes3_$TAG
exit 0
