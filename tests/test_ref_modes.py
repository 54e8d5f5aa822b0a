"""Online modes whose error behaviour mirrors the reference's (CPU): the
outcome the reference itself produced (tests/golden/ref_modes.npz, written by
make_golden._run_modes through the reference) against what the device path's
host side and the oracle do before any GPU work."""
import numpy as np
import pytest

from _util import make_case_params


def test_batch_estimates_init_raises_like_the_reference(golden_dir):
    from danse_amd.engine import init_scm_slices
    from oracle import danse_ref_cpu as O
    from danse_amd.scene import make_scene
    from golden_cases import REF_MODES_CASE
    g = dict(np.load(golden_dir / 'ref_modes.npz', allow_pickle=False))
    ref = str(g['batch_estimates'])
    etype, msg = ref.split(': ', 1)
    assert etype == 'TypeError'
    case = dict(name='x', M=[2, 3], dur=2.0, seed=5,
                danse=dict(REF_MODES_CASE['base'], nodeUpdating='asy', covMatInitType='batch_estimates'))
    dp, wp = make_case_params(case)
    with pytest.raises(TypeError, match=msg.replace("'", '.')):
        init_scm_slices(dp, 5, 2, 513)
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'])
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    with pytest.raises(TypeError, match=msg.replace("'", '.')):
        O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive)
