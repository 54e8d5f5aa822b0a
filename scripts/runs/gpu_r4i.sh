#!/bin/bash
# round 4: wide classes (KATs at D = 96 / 256, best-perf at sum(M) = 96 / 256),
# scene conv/VAD + condition numbers vs the reference, the dist tests, then
# the E battery bench over the L grid
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "kat or best_perf" > gpurun_out/r4i/pytest_wide.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error| w \{" gpurun_out/r4i/pytest_wide.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scene.py tests/test_gpu_engine_modes.py tests/test_gpu_dist.py -k "scene or condition or dist or rccl or shard or dxcp" > gpurun_out/r4i/pytest_r4d.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4i/pytest_r4d.log | tail -30
[ $rc -ne 0 ] && exit $rc
for L in 1 16 64 512; do
  extra="--no-cpu-baseline"
  [ "$L" = "1" ] && extra="--cpu-seconds 10"
  timeout -k 10 300 python -u bench.py --workload E_comp --L $L --scenes 512 --scene-gen device --steps 5 --warmup 1 --no-traffic $extra > gpurun_out/r4i/E_comp_L$L.log 2>&1 || { echo "bench L=$L failed rc=$?"; tail -5 gpurun_out/r4i/E_comp_L$L.log; exit 1; }
  tail -1 gpurun_out/r4i/E_comp_L$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('E_comp L=$L', round(d['value']/1e9,3), 'G FU/s', round(d['ms_per_step'],2), 'ms/step scene_gen_s', d.get('scene_gen_s'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
# broadcast-kernel ablation at N2 (timing only: results are wrong with a
# nonzero mask): 1 no analyses, 2 no z synthesis/analysis, 4 no estimate
# synthesis, 64 no FFTs
for ab in 0 1 2 4 64; do
  DANSE_BCAST_ABLATE=$ab timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i/ab$ab -o kt -- python bench.py --workload N2 --steps 1 --warmup 0 --no-traffic --no-cpu-baseline > gpurun_out/r4i/ab$ab.log 2>&1 || { echo "ablation $ab failed"; exit 1; }
  echo "ablate $ab: $(grep bcast_kernel $(find gpurun_out/r4i/ab$ab -name '*kernel_stats.csv' | head -1) | cut -d, -f2-4)"
done
