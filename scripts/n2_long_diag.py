"""Diagnostics of the N2 long-run parity case (tests/test_gpu_engine_modes.py
test_headline_shape_K32x8_D39_long_run_vs_oracle): the float64 oracle once,
then the device under engine switches (default; DANSE_NO_WARM=1: no warm
Lanczos; DANSE_NO_R1=1: no rank-one factor records), each compared with the
oracle per (node, bin, post-gate round): error percentiles, outlier counts and
the worst entries.  Oracle outputs are cached in /tmp between invocations."""
from __future__ import annotations

import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tests'))
sys.path.insert(0, str(ROOT / 'tests' / 'golden'))


def main():
    from danse_amd.engine import DanseEngine
    from danse_amd.scene import make_scene
    from oracle import danse_ref_cpu as O
    from _util import make_case_params
    from golden_cases import BATTERY
    post = int(os.environ.get('N2_POST', '40'))
    configs = (os.environ.get('N2_CONFIGS') or 'default,DANSE_NO_WARM,DANSE_NO_R1').split(',')
    case = dict(name='online_N2_K32x8_long', M=[8] * 32, dur=4.5, seed=41, danse=dict(BATTERY, nodeUpdating='asy'))
    dp, wp = make_case_params(case)
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'], pauseDuration=0.9)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    K = 32
    runs = {}
    for cfg in configs:
        for k in ('DANSE_NO_WARM', 'DANSE_NO_R1'):
            os.environ.pop(k, None)
        if cfg != 'default':
            os.environ[cfg] = '1'
        eng = DanseEngine([sc], dp)
        t = time.time()
        eng.run()
        dv = eng.outputs()[0]
        runs[cfg] = (dv, eng.lanczos_stats())
        eng.close()
        print(f'# device {cfg}: {time.time() - t:.1f} s', flush=True)
    dv0 = runs[configs[0]][0]
    R0 = int(np.max(dv0.startRound)) + post
    O.set_workers(min(16, max(2, len(os.sched_getaffinity(0)))))
    try:
        ov = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive, maxRounds=R0)
        ov.progressEvery = 8
        ov.run()
    finally:
        O.set_workers(0)
    for cfg, (dv, lz) in runs.items():
        errs = []
        for k in range(K):
            s0 = int(ov.startRound[k])
            wd, wo = dv.wTilde[k][:, s0 + 1:R0 + 1], ov.wTilde[k][:, s0 + 1:R0 + 1]
            e = np.linalg.norm(wd - wo, axis=-1) / np.maximum(np.linalg.norm(wo, axis=-1), 1e-30)   # [F][rounds]
            errs.append(e)
        E = np.stack(errs)   # [K][F][rounds]
        flat = E.ravel()
        print(f'{cfg}: median {np.median(flat):.3g} p99 {np.percentile(flat, 99):.3g} p99.9 '
              f'{np.percentile(flat, 99.9):.3g} max {flat.max():.3g}; >1e-4: {int((flat > 1e-4).sum())}, '
              f'>1e-3: {int((flat > 1e-3).sum())} of {flat.size}; lanczos sent back {int(lz[:, 1].sum())}')
        # the same errors relative to the bin's median oracle filter norm over
        # the window (a filter that passes near zero -- lambda_1 near 1 makes
        # (1 - 1/lambda_1) cancel -- inflates the per-entry relative error)
        Nrm = np.stack([np.linalg.norm(ov.wTilde[k][:, int(ov.startRound[k]) + 1:R0 + 1], axis=-1) for k in range(K)])
        med = np.median(Nrm, axis=-1, keepdims=True)
        En = E * Nrm / np.maximum(med, 1e-30)
        fn = En.ravel()
        print(f'{cfg} (normalised by the bin median norm): median {np.median(fn):.3g} p99 {np.percentile(fn, 99):.3g} '
              f'max {fn.max():.3g}; >1e-3: {int((fn > 1e-3).sum())}')
        idx = np.argsort(flat)[::-1][:12]
        for i in idx:
            k, f, r = np.unravel_index(i, E.shape)
            print(f'   k {k:2d} f {f:3d} post-gate round {r:2d}: {E[k, f, r]:.3g} norm/median {Nrm[k, f, r] / med[k, f, 0]:.3g} '
                  f'(same bin, rounds: {" ".join(f"{x:.1e}" for x in E[k, f, max(0, r - 3):r + 4])})')
        sys.stdout.flush()


if __name__ == '__main__':
    main()
