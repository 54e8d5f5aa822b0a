#!/bin/bash
# round 4: Lanczos v2 (one-pass CGS, unrolled) -- 2d-class parity, N2 / C /
# B timing warm vs no-warm, SQ counters of the N2 update kernel
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine_modes.py -k "headline or large_D or shape or kat_gevd or resident_B" > gpurun_out/r4g/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed| w \{|resident w" gpurun_out/r4g/pytest.log | tail -40
[ $rc -ne 0 ] && exit $rc
for W in N2 C; do for v in warm nowarm; do
  if [ $v = nowarm ]; then export DANSE_NO_WARM=1; else unset DANSE_NO_WARM; fi
  timeout -k 10 300 python -u bench.py --workload $W --steps 4 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/r4g/bench_${W}_$v.log 2>&1 || { echo "bench $W $v failed"; tail -5 gpurun_out/r4g/bench_${W}_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4g/bench_${W}_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$W $v', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],1), 'ms', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us', r['frac'])"
done; done
unset DANSE_NO_WARM
timeout -k 10 300 python -u bench.py --workload B --scenes 1 --resident --steps 5 --warmup 2 --no-extra --no-traffic --no-cpu-baseline > gpurun_out/r4g/bench_Bres.log 2>&1 || { echo "bench Bres failed"; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4g/bench_Bres.log').read().strip().splitlines()[-1]); print('B S1 resident', round(d['value']/1e6,1), 'M FU/s', round(d['ms_per_step'],2), 'ms')"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d gpurun_out/r4g/pmcN2 -o pmc --output-format csv -- python bench.py --workload N2 --steps 1 --warmup 0 --no-traffic --no-cpu-baseline > gpurun_out/r4g/pmcN2.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r4g/pmcN2.log; exit 1; }
python scripts/pmc_rounds.py $(find gpurun_out/r4g/pmcN2 -name "*counter_collection.csv" | head -1) update_kernel_2d
