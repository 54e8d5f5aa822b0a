#!/bin/bash
# round 4: scene conv/VAD vs the reference, condition numbers vs the
# reference fixture, then the E battery bench over the L grid (512 scenes /
# GPU, device scene generation timed beside the step)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/benchE_r4d
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scene.py tests/test_gpu_engine_modes.py -k "scene or condition" > gpurun_out/pytest_r4d.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|mismatch|vs the reference|cond error" gpurun_out/pytest_r4d.log | tail -20
[ $rc -ne 0 ] && exit $rc
for L in 1 2 4 8 16 32 64 128 256 512; do
  extra="--no-cpu-baseline"
  [ "$L" = "1" ] || [ "$L" = "512" ] && extra="--cpu-seconds 10"
  timeout -k 10 300 python -u bench.py --workload E_comp --L $L --scenes 512 --scene-gen device --steps 5 --warmup 1 --no-traffic $extra > gpurun_out/benchE_r4d/E_comp_L$L.log 2>&1 || { echo "bench L=$L failed rc=$?"; tail -5 gpurun_out/benchE_r4d/E_comp_L$L.log; exit 1; }
  tail -1 gpurun_out/benchE_r4d/E_comp_L$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('E_comp L=$L', round(d['value']/1e9,3), 'G FU/s', round(d['ms_per_step'],2), 'ms/step scene_gen_s', d.get('scene_gen_s'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
for L in 1 16 512; do
  timeout -k 10 300 python -u bench.py --workload E_noComp --L $L --scenes 512 --scene-gen device --steps 5 --warmup 1 --no-traffic --no-cpu-baseline > gpurun_out/benchE_r4d/E_noComp_L$L.log 2>&1 || { echo "bench noComp L=$L failed rc=$?"; tail -5 gpurun_out/benchE_r4d/E_noComp_L$L.log; exit 1; }
  tail -1 gpurun_out/benchE_r4d/E_noComp_L$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('E_noComp L=$L', round(d['value']/1e9,3), 'G FU/s', round(d['ms_per_step'],2), 'ms/step scene_gen_s', d.get('scene_gen_s'))"
done
