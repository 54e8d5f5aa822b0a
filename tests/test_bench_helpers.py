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
    AVG, SET, KEEP = bench.OP_AVG, bench.OP_SET, bench.OP_KEEP
    assert (KEEP, SET, AVG) == (0, 1, 2)
    # SURVEY §8d (c64 packed): VAD frame with a solve = B_cov + the solve's
    # read of Rnn and write of w: 1.15 KB + 0.62 KB at D = 11
    assert bench.alg_bytes_update(D, AVG, KEEP, True) == 8 * t + 8 * D + 8 + 4 * t + 8 * D == 1768
    # noise frame without a solve: Rnn read + write
    assert bench.alg_bytes_update(D, KEEP, AVG, False) == 8 * D + 8 + 8 * t
    # first frame sets the SCM: write only
    assert bench.alg_bytes_update(D, SET, KEEP, False) == 8 * D + 8 + 4 * t
    assert bench.alg_bytes_update(39, AVG, KEEP, True) == 8 * 39 * 40 + 8 * 39 + 8 + 4 * 39 * 40 + 8 * 39
    b = bench.alg_bytes_update(D, np.array([AVG, KEEP]), np.array([KEEP, AVG]), np.array([True, False]))
    assert b.shape == (2,)
    # engine storage: Ryy c64, Rnn c128 (twice the bytes), the w ring
    assert bench.storage_bytes_update(D, KEEP, AVG, False) == 8 * D + 8 + 16 * t + 16 * D
    assert bench.storage_bytes_update(D, AVG, KEEP, True) == 8 * D + 8 + 8 * t + 8 * t + 8 * D
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
