"""Diagnostics: the lean cached-C solves (kernels_2dc.hpp) against the
engine without the C cache (DANSE_NO_CCACHE=1), on the N2 long-run scene of
test_headline_shape_K32x8_D39_long_run_vs_oracle: per round the largest
per-bin relative filter difference between the two device runs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests', 'golden'))


def run(env, sc, dp):
    from danse_amd.engine import DanseEngine
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        eng = DanseEngine([sc], dp)
        eng.run()
        out = eng.outputs()[0]
        lz = eng.lanczos_stats()
        eng.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return out, lz


def main():
    from golden_cases import BATTERY
    from _util import make_case_params
    from danse_amd.scene import make_scene
    case = dict(name='n2long', M=[8] * 32, dur=4.5, seed=41, danse=dict(BATTERY, nodeUpdating='asy'))
    dp, wp = make_case_params(case)
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'], pauseDuration=0.9)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    ref, _ = run({'DANSE_NO_CCACHE': '1'}, sc, dp)
    new, lz = run({}, sc, dp)
    K = 32
    s0 = int(np.min(ref.startRound))
    R = ref.nRounds if hasattr(ref, 'nRounds') else ref.wTilde[0].shape[1] - 1
    print('starts equal', np.array_equal(ref.startRound, new.startRound), 's0', s0, flush=True)
    vad = np.array([nd.vadPerFrame[:R] for nd in sc.wasn])
    for r in range(s0, min(s0 + 60, R)):
        e = []
        for k in range(K):
            a = new.wTilde[k][:, r + 1]
            b = ref.wTilde[k][:, r + 1]
            e.append(np.max(np.linalg.norm(a - b, axis=-1) / np.maximum(np.linalg.norm(b, axis=-1), 1e-30)))
        e = np.array(e)
        print(r, 'vad', int(vad[:, r].sum()), 'max', '%.2e' % e.max(), 'median', '%.2e' % np.median(e),
              'worst node', int(np.argmax(e)), 'lz', lz[r].tolist(), flush=True)


if __name__ == '__main__':
    main()
