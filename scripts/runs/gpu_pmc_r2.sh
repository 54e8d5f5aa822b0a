#!/bin/bash
# PMC counters for the update kernels (each pass its own run, time-limited):
# wave / instruction / stall counters, then HBM bytes (FETCH_SIZE, WRITE_SIZE).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
ARGS=${ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --no-traffic --scenes 31"}
i=0
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $PASS --kernel-trace -d gpurun_out/pmc_${TAG}_$i -o pmc --output-format csv -- python bench.py $ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
python3 scripts/pmc_table.py gpurun_out/pmc_${TAG}_[0-9]* > gpurun_out/pmc_${TAG}_summary.txt 2>&1
cat gpurun_out/pmc_${TAG}_summary.txt | head -60
