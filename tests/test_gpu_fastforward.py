"""The pre-solve prefix fast-forward (csrc/span.hpp) against
the per-round recursion (DANSE_NO_FF=1), ``-m gpu``: the same filters,
estimates and start rounds.  The span kernel's arithmetic is the
recursion-only kernels' entry by entry, but the compiler contracts the
multiply-adds of the two kernels differently: the outputs differ at float32
rounding (d 1.0-1.8e-7 relative on MI355X, gpurun_out/pytest_ff.log of round
5), bounded here at 1e-5."""
import os

import numpy as np
import pytest

from golden_cases import ONLINE_CASES, BATTERY
from _util import make_case_params, make_case_scene

pytestmark = pytest.mark.gpu

pytest.importorskip('torch')

CASES = [c for c in ONLINE_CASES if c['name'] in ('online_B_k4m3_asy', 'online_B_k4m3_seq', 'online_ragged_asy_r2')]
CASES.append(dict(name='online_K8x4_asy_4s', M=[4] * 8, dur=4.0, seed=31, danse=dict(BATTERY, nodeUpdating='asy')))
# the row-per-lane classes (update_kernel_big: the MWF above D = 12, the GEVD
# of D 49..64) without the first-frame basis: the random init is then
# averaged from round 0, so a prefix round that ran the recursion in place
# AND was replayed by span_rec_kernel would decay the SCMs twice
CASES.append(dict(name='online_big_D20_mwf_nobasis', M=[17, 4, 4, 5], dur=3.0, seed=23,
                  danse=dict(BATTERY, nodeUpdating='asy', performGEVD=False, use1stFrameAsBasis=False)))
CASES.append(dict(name='online_big_D51_nobasis', M=[48, 2, 2, 2], dur=4.0, seed=25,
                  danse=dict(BATTERY, nodeUpdating='asy', use1stFrameAsBasis=False)))


def _run(case, ff):
    from danse_amd.core import danse_multi
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    old = os.environ.get('DANSE_NO_FF')
    if ff:
        os.environ.pop('DANSE_NO_FF', None)
    else:
        os.environ['DANSE_NO_FF'] = '1'
    try:
        return danse_multi([sc], dp)[0]
    finally:
        if old is None:
            os.environ.pop('DANSE_NO_FF', None)
        else:
            os.environ['DANSE_NO_FF'] = old


@pytest.mark.parametrize('case', CASES, ids=lambda c: c['name'])
def test_prefix_fast_forward_matches_per_round_recursion(case):
    a = _run(case, True)
    b = _run(case, False)
    assert np.array_equal(a.startRound, b.startRound)
    K = len(case['M'])
    for k in range(K):
        s0 = int(b.startRound[k])
        wa, wb = a.wTilde[k][:, s0 + 1:], b.wTilde[k][:, s0 + 1:]
        err = np.max(np.abs(wa - wb)) / max(np.max(np.abs(wb)), 1e-30)
        assert err <= 1e-5, (case['name'], k, err)
    de = np.max(np.abs(a.d - b.d)) / max(np.max(np.abs(b.d)), 1e-30)
    print(case['name'], 'd', de, 'identical', np.array_equal(a.d, b.d))
    assert de <= 1e-5
