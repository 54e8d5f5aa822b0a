#!/usr/bin/env python3
"""Calibrate bench.py's CPU leg (THIS CONTAINER ONLY: it imports the reference
through tests/golden/_refharness.py; nothing on the GPU box runs it).

Runs, on the same synthetic scene and battery settings:
  1. the reference's own online DANSE (danse_toolbox d_core.danse) end to end,
  2. the float64 oracle (oracle/danse_ref_cpu.py) end to end,
  3. bench.cpu_baseline's bounded-sample projection of the oracle's whole run,
and prints the three wall times (and FU/s) as one JSON line, so the oracle
("port") can be checked against the reference rate (SURVEY §8d asks for
+-20%) and the projection against the oracle's real run.

    python scripts/calibrate_cpu_baseline.py [--K 8] [--M 4] [--dur 4] [--seq]

BLAS threads are whatever the environment gives (set OPENBLAS_NUM_THREADS to
compare thread counts); the same setting applies to all three legs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tests' / 'golden'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--K', type=int, default=8)
    ap.add_argument('--M', type=int, default=4)
    ap.add_argument('--dur', type=float, default=4.0)
    ap.add_argument('--seq', action='store_true')
    ap.add_argument('--no-ref', action='store_true')
    args = ap.parse_args()
    import bench
    from danse_amd.scene import make_scene
    from oracle import danse_ref_cpu as O
    M = [args.M] * args.K
    upd = 'seq' if args.seq else 'asy'
    wl = dict(M=M, dur=args.dur, nodeUpdating=upd)
    dp, wp = bench._wl_params(wl)
    sc = make_scene(M, sigDur=args.dur, seed=1000)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    K, F = len(M), dp.DFTsize // 2 + 1
    out = {'K': K, 'M': args.M, 'dur': args.dur, 'nodeUpdating': upd,
           'threads_env': {k: os.environ.get(k) for k in ('OPENBLAS_NUM_THREADS', 'OMP_NUM_THREADS')}}

    t = time.perf_counter()
    ov = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive)
    ov.run()
    out['oracle_s'] = time.perf_counter() - t
    R = int(np.max(ov.i))
    out['rounds'] = R
    out['oracle_FUps'] = K * F * R / out['oracle_s']

    cb = bench.cpu_baseline(M, wl, dp, wp, 15.0, R)
    out['projection_s'] = cb['projected_run_s']
    out['projection_FUps'] = cb['value']
    out['projection_method'] = cb['sample']

    if not args.no_ref:
        import _refharness as H
        from golden_cases import BATTERY, _d
        ns = H.load()
        p = H.make_params(ns, M, **_d(BATTERY, nodeUpdating=upd, startComputeMetricsAt='after_5s'))
        w = H.to_ref_wasn(ns, sc)
        p, w = H.prep(ns, p, w)
        t = time.perf_counter()
        ns.core.danse(w, p.danseParams)
        out['reference_s'] = time.perf_counter() - t
        out['reference_FUps'] = K * F * R / out['reference_s']
        out['oracle_over_reference_rate'] = out['oracle_FUps'] / out['reference_FUps']
    out['projection_over_oracle_time'] = out['projection_s'] / out['oracle_s']
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
