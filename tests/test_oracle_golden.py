"""The CPU oracle (oracle/danse_ref_cpu.py) against golden vectors produced by
the reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from golden_cases import ONLINE_CASES, BATCH_CASES, SRO_EVENT_CASES, KAT_CASES, DXCP_CASES, TZ_CASES, kat_inputs
from golden_cases import BESTPERF_CASES, SCENE_CASES, scene_inputs, COND_CASES
from danse_amd.scene import scene_digest
from danse_amd.scheduler import initialize_events
from oracle import danse_ref_cpu as O
from _util import make_case_params, make_case_scene, rel_err

TOL = 1e-10


def _load(golden_dir, name):
    return dict(np.load(golden_dir / f'{name}.npz', allow_pickle=False))


@pytest.mark.parametrize('case', ONLINE_CASES, ids=[c['name'] for c in ONLINE_CASES])
def test_online_oracle_matches_reference(case, golden_dir):
    g = _load(golden_dir, case['name'])
    sc = make_case_scene(case)
    assert scene_digest(sc) == str(g['digest']), 'regenerated scene differs from the one the fixture was made on'
    dp, wp = make_case_params(case)
    dv = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive)
    every = 16
    assert rel_err(dv.d, g['d']) < TOL
    if np.all(np.isnan(g['dhat'])):   # desSigProcessingType 'conv': dhatCurr = None
        assert np.all(np.isnan(dv.dhat[:, ::every, :]))
    else:
        assert rel_err(dv.dhat[:, ::every, :], g['dhat']) < TOL
    for k in range(len(case['M'])):
        assert rel_err(dv.wTilde[k][:, ::every, :], g[f'w_{k}']) < TOL
        if f'wExt_{k}' in g:
            assert rel_err(dv.wTildeExt[k][:, ::every, :], g[f'wExt_{k}']) < TOL
        if f'z_{k}' in g:
            assert rel_err(dv.zFullTD[k], g[f'z_{k}']) < TOL
        if f'wLocal_{k}' in g:
            assert rel_err(dv.wLocal[k][:, ::every, :], g[f'wLocal_{k}']) < TOL
        if f'wCentr_{k}' in g:
            assert rel_err(dv.wCentr[k][:, ::every, :], g[f'wCentr_{k}']) < TOL
    for nm in ['dLocal', 'dCentr', 'dSSBC']:
        if nm in g:
            assert rel_err(getattr(dv, nm), g[nm]) < TOL
    assert np.array_equal(np.array([s.start for s in dv.danse]), g['startUpdates'])
    assert np.array_equal(dv.nInternalFilterUps, g['nInternalFilterUps'])
    if case.get('snr_replay'):
        sigs = O.generate_signals_for_snr_computation(sc, dp, dv, vadMinProp=wp.vadMinProportionActive)
        assert rel_err(sigs['n'], g['snr_n']) < TOL
        assert rel_err(sigs['s'], g['snr_s']) < TOL


@pytest.mark.parametrize('case', BATCH_CASES, ids=[c['name'] for c in BATCH_CASES])
def test_batch_oracle_matches_reference(case, golden_dir):
    g = _load(golden_dir, case['name'])
    sc = make_case_scene(case)
    assert scene_digest(sc) == str(g['digest'])
    dp, wp = make_case_params(case)
    bv = O.danse_batch(sc, dp, vadMinProp=wp.vadMinProportionActive)
    assert rel_err(bv.d, g['d']) < TOL
    assert rel_err(np.array(bv.mmseCost, dtype=float), g['mmseCost']) < TOL
    for k in range(len(case['M'])):
        nb = case['danse']['maxBatchUpdates'] + 1
        assert rel_err(bv.wTilde[k][:, :nb, :], g[f'w_{k}']) < TOL
    for fam in ('Centr', 'Local'):
        if f'd{fam}' in g:
            assert rel_err(getattr(bv, f'd{fam}'), g[f'd{fam}']) < TOL
            assert rel_err(np.array(getattr(bv, f'mmseCost{fam}')), g[f'mmseCost{fam}']) < TOL
            for k in range(len(case['M'])):
                assert rel_err(getattr(bv, f'w{fam}')[k][:, :2, :], g[f'w{fam}_{k}']) < TOL


@pytest.mark.parametrize('case', BESTPERF_CASES, ids=[c['name'] for c in BESTPERF_CASES])
def test_best_perf_oracle_matches_reference(case, golden_dir):
    """get_best_perf (d_core.py:602-627) and its noise-only / speech-only
    replays with the recorded centralised filters."""
    import copy
    from danse_amd.params import PreComputedFilters
    g = _load(golden_dir, case['name'])
    sc = make_case_scene(case)
    assert scene_digest(sc) == str(g['digest'])
    dp, wp = make_case_params(case)
    bp = O.get_best_perf(sc, dp, vadMinProp=wp.vadMinProportionActive)
    assert rel_err(bp.dCentr, g['dCentr']) < TOL
    assert rel_err(np.array(bp.mmseCostCentr), g['mmseCostCentr']) < TOL
    for k in range(len(case['M'])):
        assert rel_err(bp.wCentr[k][:, :2, :], g[f'wCentr_{k}']) < TOL
    pU = copy.deepcopy(dp)
    for purpose in ('noise-only', 'speech-only'):
        pU.preGivenFilters = PreComputedFilters(active=True, purpose=purpose)
        o = O.get_best_perf(sc, pU, wCentr=bp.wCentr, vadMinProp=wp.vadMinProportionActive)
        assert rel_err(o.dCentr, g[f'dCentr_{purpose[0]}']) < TOL


@pytest.mark.parametrize('case', SRO_EVENT_CASES, ids=[c['name'] for c in SRO_EVENT_CASES])
def test_scheduler_matches_reference(case, golden_dir):
    """Host event scheduler (danse_amd/scheduler.py) vs the reference's
    initialize_events, including SRO clocks (quirks Q3, Q13)."""
    g = _load(golden_dir, case['name'])
    sc = make_case_scene(dict(case, seed=0), SROperNode=case['sros'])
    dp, wp = make_case_params(case, SROperNode=case['sros'])
    ev, fs = initialize_events([n.timeStamps for n in sc.wasn], [n.fs for n in sc.wasn], dp,
                               [n.neighborsIdx for n in sc.wasn])
    rows = [(e.t, int(e.nodes[ii]), 0 if e.type[ii] == 'bc' else 1, int(e.bypassUpdate[ii]))
            for e in ev for ii in range(e.nEvents)]
    ref = g['events']
    assert len(ev) == int(g['n_instants'])
    assert len(rows) == len(ref)
    got = np.array(rows, dtype=ref.dtype)
    for f in ref.dtype.names:
        assert np.array_equal(got[f], ref[f]), f
    assert np.array_equal(fs, g['fs'])


@pytest.mark.parametrize('case', KAT_CASES, ids=[c['name'] for c in KAT_CASES])
def test_filter_update_kat(case, golden_dir):
    g = _load(golden_dir, case['name'])
    Ryy, Rnn = kat_inputs(case)
    fn = O.update_w_gevd if case['gevd'] else O.update_w
    w = fn(Ryy, Rnn, refSensorIdx=case['ref'], rank=case['rank'])
    assert rel_err(w, g['w']) < 1e-12


@pytest.mark.parametrize('case', DXCP_CASES, ids=[c['name'] for c in DXCP_CASES])
def test_dxcp_oracle_matches_reference(case, golden_dir):
    """DXCP-PhaT restatement (oracle/dxcp_ref.py) against the reference's
    DXCPPhaT run on the same two-channel input: identical per-frame SRO and
    STO estimates."""
    import warnings
    from golden_cases import dxcp_inputs
    from oracle import dxcp_ref as D
    g = _load(golden_dir, case['name'])
    x1, x2 = dxcp_inputs(case)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', DeprecationWarning)
        sro, sto = D.run(x1, x2)
    assert np.max(np.abs(sro - g['sro'])) <= 1e-9
    assert np.max(np.abs(sto - g['sto'])) <= 1e-9
    assert abs(sro[-1] - case['sro']) < 1.0     # converged estimate


@pytest.mark.parametrize('case', TZ_CASES, ids=[c['name'] for c in TZ_CASES])
def test_tz_oracle_matches_reference(case, golden_dir):
    """T(z) few-samples restatement (oracle/tz_ref.py) against the
    reference's dist_fct_approx + danse_compression_few_samples; the closed
    form IR (the one the device computes) against the literal restatement."""
    from golden_cases import tz_inputs
    from oracle import tz_ref as T
    g = _load(golden_dir, case['name'])
    wHat, yq, h, f, wPrev = tz_inputs(case)
    z, wIR = T.danse_compression_few_samples(yq, wHat, case['L'], wPrev, h, f, case['Ns'],
                                             updateBroadcastFilter=case['update'])
    assert rel_err(wIR, g['wIR']) < TOL
    assert rel_err(z, g['z']) < TOL
    if case['update']:
        assert rel_err(T.dist_fct_approx_closed(wHat, h, f, case['Ns']), g['wIR']) < TOL


@pytest.mark.parametrize('case', __import__('golden_cases').METRIC_CASES, ids=lambda c: c['name'])
def test_metrics_oracle_vs_reference(case, golden_dir):
    """oracle/metrics_ref.py (get_snr, get_fwsnrseg) against the reference's
    own d_eval functions run on the same inputs."""
    from golden_cases import metric_inputs
    from oracle import metrics_ref as MR
    g = np.load(golden_dir / f"{case['name']}.npz")
    clean, enh, s, n, vad = metric_inputs(case)
    kw = {k: case[k] for k in ('frameLen', 'overlap', 'gamma') if k in case}
    fw = MR.get_fwsnrseg(clean, enh, case['fs'], **kw)
    assert fw.shape == g['fw'].shape
    assert np.max(np.abs(fw - g['fw'])) <= 1e-9
    assert np.allclose(MR.get_snr(s, n, vad), g['snr'], rtol=1e-12, atol=1e-12)
    assert np.allclose(MR.get_snr(s, n, vad, bypassVADuse=True), g['snrAll'], rtol=1e-12, atol=1e-12)
    assert np.allclose(MR.get_snr(s[:, 0], n[:, 0], vad[:, 0]), g['snr1'], rtol=1e-12, atol=1e-12)
    if case['same']:
        assert np.any(g['fw'] == 35.0)   # identical frames clip at 35 dB


def test_get_metrics_quirks_vs_reference(golden_dir):
    """The reference's get_metrics ('snr', 'fwSNRseg'): SNR over the whole
    trimmed signal (bypassVADuse hard-coded True) and fwSNRseg with the
    positional gamma landing in `overlap` (d_eval.py:205,236-242), restated
    with the oracle functions."""
    from golden_cases import GETMETRICS_CASE as case, get_metrics_inputs
    from oracle import metrics_ref as MR
    g = np.load(golden_dir / f"{case['name']}.npz")
    kw = get_metrics_inputs(case)
    sl = slice(case['startIdx'], case['endIdx'])
    fs = case['fs']
    c = kw['clean'][sl]
    assert np.isclose(MR.get_snr(kw['clean'][sl], kw['noiseOnly'][sl]), g['snr_before'], rtol=1e-12)
    assert np.isclose(MR.get_snr(kw['filtSpeech'][sl], kw['filtNoise'][sl]), g['snr_after'], rtol=1e-12)
    assert np.isclose(MR.get_snr(kw['filtSpeech_c'][sl], kw['filtNoise_c'][sl]), g['snr_afterCentr'], rtol=1e-12)
    enh = kw['filtSpeech'][sl] + kw['filtNoise'][sl]
    for fld, e in (('before', kw['noisy'][sl]), ('after', enh), ('afterCentr', kw['enhan_c'][sl]),
                   ('afterLocal', kw['enhan_l'][sl])):
        v = np.mean(MR.get_fwsnrseg(c, e, fs, 0.03, 0.2))   # overlap = gamma = 0.2
        assert abs(v - g[f'fwSNRseg_{fld}']) <= 1e-9, fld


from golden_cases import STOI_CASES, stoi_inputs  # noqa: E402


@pytest.mark.parametrize('case', STOI_CASES, ids=[c['name'] for c in STOI_CASES])
def test_stoi_oracle_vs_reference(case, golden_dir):
    """oracle/metrics_ref.stoi against mypystoi (stoi_any_fs at 10 kHz, stoi
    at 16 kHz), both float64 (the reference adds EPS-scale noise in eSTOI)."""
    from oracle import metrics_ref as MR
    g = _load(golden_dir, case['name'])
    x, y = stoi_inputs(case)
    assert abs(MR.stoi(x, y, case['fs'], extended=True) - float(g['estoi'])) <= 1e-12
    assert abs(MR.stoi(x, y, case['fs'], extended=False) - float(g['stoi'])) <= 1e-12


from golden_cases import CLDXCP_CASES, cldxcp_acs  # noqa: E402


@pytest.mark.parametrize('case', CLDXCP_CASES, ids=[c['name'] for c in CLDXCP_CASES])
def test_cl_dxcp_oracle_matches_reference(case, golden_dir):
    """oracle/dxcp_ref.run_closed_loop against the reference's CL_DXCPPhaT
    (sro_estimation.py:12-72): bit for bit."""
    import warnings
    from golden_cases import dxcp_inputs
    from oracle import dxcp_ref as D
    g = _load(golden_dir, case['name'])
    x1, x2 = dxcp_inputs(case)
    n = len(x1) // 2048
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', DeprecationWarning)
        out, zi = D.run_closed_loop(x1, x2, case['startDelay'], cldxcp_acs(case, n))
    assert np.array_equal(out, g['out'])
    assert np.array_equal(zi[::5], g['zi'])


def test_gevd_pool_bit_identical(golden_dir):
    """The oracle's per-bin eigh spread over worker processes
    (oracle/_gevd_pool.py, used by the heavy parity tests) gives the serial
    loop's filters bit for bit, on the filter-update KAT inputs."""
    case = next(c for c in KAT_CASES if c['name'] == 'kat_gevd_D19_r1')
    Ryy, Rnn = kat_inputs(case)
    serial = O.update_w_gevd(Ryy, Rnn, 0, 2)
    O.set_workers(3)
    try:
        pooled = O.update_w_gevd(Ryy, Rnn, 0, 2)
    finally:
        O.set_workers(0)
    assert np.array_equal(serial, pooled)


@pytest.mark.parametrize('case', SCENE_CASES, ids=[c['name'] for c in SCENE_CASES])
def test_scene_vad_conv_vs_reference(case, golden_dir):
    """oracle/scene_ref.py (the device scene generator's checker) against the
    reference's get_vad on injected inputs: wet signals (fftconvolve) to
    1e-12, the per-sample VAD of each node's reference sensor exactly, on the
    float64 wet signals and on their float32 rounding."""
    from oracle import scene_ref as SR
    g = _load(golden_dir, case['name'])
    x, h = scene_inputs(case)
    assert np.array_equal(x, g['x']) and np.array_equal(h, g['h'])
    wet = np.stack([SR.wet_signal(x, hc) for hc in h])
    assert rel_err(wet, g['wet']) < 1e-12
    ref = np.cumsum([0] + list(case['M']))[:-1]
    for j, b in enumerate(ref):
        v = SR.energy_vad(g['wet'][b], case['fs'], case['vadWinLength'], case['vadEnergyDecrease_dB'])
        assert np.array_equal(v, g['vad'][j]), j
        w32 = g['wet'][b].astype(np.float32).astype(np.float64)
        v32 = SR.energy_vad(w32, case['fs'], case['vadWinLength'], case['vadEnergyDecrease_dB'])
        assert np.array_equal(v32, g['vad32'][j]), j
        assert 0.05 < v.mean() < 0.95


@pytest.mark.parametrize('case', COND_CASES, ids=[c['name'] for c in COND_CASES])
def test_condition_numbers_oracle_vs_reference(case, golden_dir):
    """The oracle's condNumbers (ConditionNumbers, d_classes.py:19-130,
    2126-2186) against the reference's own: the same saved iterations, and
    np.linalg.cond of the same float64 SCMs (<= 1e-6 relative where the
    reference's value is below 1e8; the rank-one first-frame basis gives
    ~1e17, where both must be numerically singular)."""
    g = _load(golden_dir, case['name'])
    sc = make_case_scene(case)
    assert scene_digest(sc) == str(g['digest'])
    dp, wp = make_case_params(case)
    ov = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive)
    cn = ov.condNumbers
    for k in range(len(case['M'])):
        for fam in ('DANSE', 'Local'):
            it = np.asarray(getattr(cn, f'iter_cn_Ryy{fam}')[k])
            assert np.array_equal(it, g[f'iter_{fam}_{k}']), (fam, k)
            a, b = np.asarray(getattr(cn, f'cn_Ryy{fam}')[k]), g[f'cn_{fam}_{k}']
            assert a.shape == b.shape
            ok = b < 1e8
            assert np.max(np.abs(a[ok] - b[ok]) / b[ok]) <= 1e-6, (fam, k)
            assert np.all(a[~ok] > 1e10), (fam, k)


def test_multi_ref_filters_bit_identical():
    """The oracle's one-decomposition centralised filters (update_w_gevd_refs /
    update_w_refs, used by get_best_perf for all nodes' references) equal
    separate update_w_gevd / update_w calls bit for bit."""
    case = next(c for c in KAT_CASES if c['name'] == 'kat_gevd_D19_r1')
    Ryy, Rnn = kat_inputs(case)
    refs = [0, 3, 18]
    for rank in (1, 2):
        many = O.update_w_gevd_refs(Ryy, Rnn, refs, rank=rank)
        for r, w in zip(refs, many):
            assert np.array_equal(w, O.update_w_gevd(Ryy, Rnn, r, rank))
    many = O.update_w_refs(Ryy, Rnn, refs)
    for r, w in zip(refs, many):
        assert np.array_equal(w, O.update_w(Ryy, Rnn, r))


def test_oracle_centralised_restriction_exact():
    """The oracle's test-side restriction for the wide centralised family
    (skipDanse / centrBins / centrNodes, exact in synchronous wholeChunk runs:
    the centralised vector is the nodes' raw frames) gives the full oracle's
    centralised filters on the kept nodes and bins, and its start rounds --
    the full oracle being pinned by the reference fixture of the case."""
    from oracle import danse_ref_cpu as O
    case = next(c for c in ONLINE_CASES if c['name'] == 'online_ragged_asy_r2')
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    full = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive).run()
    bins = [0, 7, 100, 512]
    sub = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive, skipDanse=True, centrBins=bins,
                        centrNodes=[1]).run()
    assert sub.startRoundCentr[1] == full.startRoundCentr[1] >= 0
    assert np.array_equal(sub.centr[1].w, full.centr[1].w[bins])
