"""CPU tests of bench.py's accounting: algorithmic bytes / flops per update
launch, the gate rounds its CPU leg projects with (must equal the oracle's
startRound) and the cpu_baseline record (SURVEY §8d fields)."""
import numpy as np

import bench
from danse_amd.scene import make_scene
from oracle import danse_ref_cpu as O


def test_alg_bytes_flops():
    D = 11
    t = D * (D + 1)
    # VAD frame with a solve: Ryy r+w (c64) + read Rnn (c128) + y, w, dhat
    assert bench.alg_bytes_update(D, 1, 0, True) == 16 * D + 8 + 8 * t + 8 * t
    # noise frame without a solve: Rnn r+w (c128)
    assert bench.alg_bytes_update(D, 0, 1, False) == 16 * D + 8 + 16 * t
    # first frame sets the SCM: write only
    assert bench.alg_bytes_update(D, 2, 0, False) == 16 * D + 8 + 4 * t
    b = bench.alg_bytes_update(D, np.array([1, 0]), np.array([0, 1]), np.array([True, False]))
    assert b.shape == (2,)
    assert bench.alg_flops_update(D, 0, 0, False) == 8 * D
    assert np.isclose(bench.alg_flops_update(39, 1, 0, True), 8 * 39 + 5 * 39 * 40 + 32 / 3 * 39 ** 3 + 12 * 39 ** 2)


def test_gate_rounds_match_oracle():
    wl = dict(M=[2, 2, 2], dur=2.0, nodeUpdating='asy')
    dp, wp = bench._wl_params(wl)
    sc = make_scene(wl['M'], sigDur=wl['dur'], seed=1000)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    D = max(wl['M']) + len(wl['M']) - 1
    ov = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive).run()
    assert np.array_equal(bench._gate_rounds(sc, D), ov.startRound)


def test_cpu_baseline_record():
    wl = dict(M=[2, 2], dur=2.0, nodeUpdating='asy')
    dp, wp = bench._wl_params(wl)
    r = bench.cpu_baseline(wl['M'], wl, dp, wp, seconds=2.0)
    for key in ('value', 'unit', 'cores', 'kind', 'sample'):
        assert key in r
    assert r['kind'] == 'port' and r['value'] > 0 and r['cores'] >= 1
    assert r['t_round_s'] > 0 and r['t_solve_node_s'] > 0
