#!/bin/bash
# Split solves (lane classes D 9..12 on 4x4 grids) + condition numbers + config C with DXCP
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3s}
DANSE_LANE_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_modes.py tests/test_gpu_parity.py -m gpu -q -s -x -k "config_B_shape or condition or sandbox or keep_history or sharded or gate or headline or config_C or large_D or init_random" --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_split_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|online_B_shape|cond error|^FAILED" gpurun_out/pytest_split_$TAG.log | tail -8
[ $rc -eq 0 ] || exit $rc
DANSE_LANE_SPLIT=1 timeout -k 10 200 python bench.py --workload B --no-cpu-baseline --no-traffic --no-extra > gpurun_out/bench_split_$TAG.log 2>&1 || exit 1
DANSE_LANE_SPLIT=0 timeout -k 10 200 python bench.py --workload B --no-cpu-baseline --no-traffic --no-extra > gpurun_out/bench_nosplit_$TAG.log 2>&1 || exit 1
python -c "
import json
for f in ['gpurun_out/bench_split_$TAG.log','gpurun_out/bench_nosplit_$TAG.log']:
    l=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(l['value']/1e6,1), round(l['ms_per_step'],2), round(l['roofline']['avg_launch_ms']*1e3,1), round(l['roofline']['frac'],3))
"
DANSE_LANE_SPLIT=1 timeout -k 10 300 python bench.py --workload N2 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/bench_N2split_$TAG.log 2>&1 || exit 1
DANSE_LANE_SPLIT=0 timeout -k 10 300 python bench.py --workload N2 --no-cpu-baseline --no-traffic --no-extra > gpurun_out/bench_N2nosplit_$TAG.log 2>&1 || exit 1
python -c "
import json
for f in ['gpurun_out/bench_N2split_$TAG.log','gpurun_out/bench_N2nosplit_$TAG.log']:
    l=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(l['value']/1e6,2), round(l['ms_per_step'],2), round(l['roofline']['avg_launch_ms']*1e3,1))
"
timeout -k 10 600 python bench.py --workload C_dxcp --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_Cdxcp_$TAG.log 2>&1; rc2=$?
tail -1 gpurun_out/bench_Cdxcp_$TAG.log | cut -c1-400
exit $rc2
