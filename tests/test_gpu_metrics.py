"""Device enhancement metrics (csrc/metrics.hip through the danse_snr /
danse_fwsnrseg C-ABI, danse_amd/metrics.py) against the float64 oracle
(oracle/metrics_ref.py) and the reference's own values (tests/golden/
metrics_*.npz).  Both sides compute in float64; tolerance 1e-8 dB per frame
(FFT and reduction order differ)."""
import numpy as np
import pytest

from golden_cases import METRIC_CASES, metric_inputs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('case', METRIC_CASES, ids=lambda c: c['name'])
def test_fwsnrseg_and_snr_vs_reference(case, golden_dir):
    from danse_amd import metrics as DM
    from oracle import metrics_ref as MR
    g = np.load(golden_dir / f"{case['name']}.npz")
    clean, enh, s, n, vad = metric_inputs(case)
    kw = {k: case[k] for k in ('frameLen', 'overlap', 'gamma') if k in case}
    fw = DM.get_fwsnrseg(clean, enh, case['fs'], **kw)
    assert fw.shape == g['fw'].shape
    e = np.max(np.abs(fw - g['fw']))
    eo = np.max(np.abs(fw - MR.get_fwsnrseg(clean, enh, case['fs'], **kw)))
    print(case['name'], 'fw vs reference', e, 'vs oracle', eo)
    assert e <= 1e-8 and eo <= 1e-8
    assert np.allclose(DM.get_snr(s, n, vad), g['snr'], rtol=1e-10, atol=1e-10)
    assert np.allclose(DM.get_snr(s, n, vad, bypassVADuse=True), g['snrAll'], rtol=1e-10, atol=1e-10)
    assert abs(DM.get_snr(s[:, 0], n[:, 0], vad[:, 0]) - float(g['snr1'])) <= 1e-10


def test_fwsnrseg_batch_mean():
    """B signal pairs in one launch: per-frame values and np.mean per pair."""
    import torch
    from danse_amd import metrics as DM
    from oracle import metrics_ref as MR
    rng = np.random.default_rng(9)
    B, T = 6, 20000
    c = rng.standard_normal((B, T))
    e = c * 0.9 + rng.standard_normal((B, T)) * np.linspace(0.01, 2.0, B)[:, None]
    per, mean = DM.fwsnrseg_batch(torch.from_numpy(c).cuda(), torch.from_numpy(e).cuda(), 16000.0)
    per, mean = per.cpu().numpy(), mean.cpu().numpy()
    for b in range(B):
        ref = MR.get_fwsnrseg(c[b], e[b], 16000.0)
        assert np.max(np.abs(per[b] - ref)) <= 1e-8
        assert abs(mean[b] - np.mean(ref)) <= 1e-9


def test_fwsnrseg_48k_large_lds():
    """fs = 48 kHz: nfft = 4096, a 96 KiB FFT workspace (above the 64 KiB
    default dynamic-LDS limit) -- against the oracle per frame."""
    import torch
    from danse_amd import metrics as DM
    from oracle import metrics_ref as MR
    rng = np.random.default_rng(48)
    B, T = 2, 48000
    c = rng.standard_normal((B, T))
    e = c * 0.8 + 0.3 * rng.standard_normal((B, T))
    per, _ = DM.fwsnrseg_batch(torch.from_numpy(c).cuda(), torch.from_numpy(e).cuda(), 48000.0)
    per = per.cpu().numpy()
    for b in range(B):
        ref = MR.get_fwsnrseg(c[b], e[b], 48000.0)
        assert per[b].shape == ref.shape
        assert np.max(np.abs(per[b] - ref)) <= 1e-8


def test_metrics_errors():
    from danse_amd import metrics as DM
    from danse_amd._lib import DanseError
    with pytest.raises(DanseError):
        DM.fwsnrseg_frames(300, 16000.0)          # shorter than one frame
    with pytest.raises(DanseError):
        DM.fwsnrseg_frames(16000, 16000.0, overlap=1.0)


def test_get_metrics_vs_reference(golden_dir):
    """danse_amd.metrics.get_metrics ('snr', 'fwSNRseg'; all fwSNRseg pairs in
    one launch) against the reference's get_metrics on the same inputs."""
    from golden_cases import GETMETRICS_CASE as case, get_metrics_inputs
    from danse_amd import metrics as DM
    g = np.load(golden_dir / f"{case['name']}.npz")
    m = DM.get_metrics(**get_metrics_inputs(case), fs=case['fs'], startIdx=case['startIdx'], endIdx=case['endIdx'],
                       metricsToPlot=['snr', 'fwSNRseg'])
    for key in ('snr', 'fwSNRseg'):
        for fld in ('before', 'after', 'diff', 'afterCentr', 'afterLocal'):
            v, r = getattr(m[key], fld), float(g[f'{key}_{fld}'])
            assert abs(v - r) <= 1e-9 * max(1.0, abs(r)), (key, fld, v, r)
    with pytest.raises(NotImplementedError):
        DM.get_metrics(**get_metrics_inputs(case), fs=case['fs'], metricsToPlot=['pesq'])


# ---- (e)STOI (csrc/stoi.hip, danse_stoi) ----------------------------------
from golden_cases import STOI_CASES, stoi_inputs, E2E_METRICS_CASE  # noqa: E402


@pytest.mark.parametrize('case', STOI_CASES, ids=lambda c: c['name'])
def test_stoi_vs_reference(case, golden_dir):
    """eSTOI and STOI against the reference's own mypystoi on the same
    inputs: stoi_any_fs at 10 kHz (no resampling), stoi() at 16 kHz (the
    Octave resampler utils.resample_oct); float64 on both sides."""
    from danse_amd import metrics as DM
    g = np.load(golden_dir / f"{case['name']}.npz")
    x, y = stoi_inputs(case)
    e = DM.stoi(x, y, case['fs'], extended=True)
    s = DM.stoi(x, y, case['fs'], extended=False)
    print(case['name'], 'estoi', e, float(g['estoi']), 'stoi', s, float(g['stoi']))
    assert abs(e - float(g['estoi'])) <= 1e-9
    assert abs(s - float(g['stoi'])) <= 1e-9


def test_stoi_batch_matches_single_calls():
    """Pairs with different silent-frame counts in one launch."""
    from danse_amd import metrics as DM
    from oracle import metrics_ref as MR
    cases = [dict(STOI_CASES[1], seed=410 + i, noise=0.1 + 0.4 * i) for i in range(4)]
    xs, ys = zip(*[stoi_inputs(c) for c in cases])
    xs, ys = np.stack(xs), np.stack(ys)
    xs[1, :30000] = 0.0   # a long silence in one pair only
    got = DM.stoi_batch(xs, ys, 16000, extended=True).cpu().numpy()
    ref = np.array([MR.stoi(a, b, 16000, extended=True) for a, b in zip(xs, ys)])
    print(got, ref)
    assert np.max(np.abs(got - ref)) <= 1e-9


def test_end_to_end_metrics_vs_reference(golden_dir):
    """North-star ΔSNR / ΔSTOI: the device DANSE run, its device SNR replays
    and the device metrics per node against the reference's own
    danse + generate_signals_for_snr_computation + get_metrics on the same
    scene (snr and fwSNRseg, before / after / diff / centralised / local,
    <= 0.01 dB), and the device eSTOI of the device estimates against the
    float64 oracle's eSTOI of the oracle's estimates (<= 0.01; the
    reference's own stoi_any_fs needs resampy at 16 kHz)."""
    from danse_amd import core, metrics as DM
    from oracle import danse_ref_cpu as O, metrics_ref as MR
    from _util import make_case_params, make_case_scene
    case = E2E_METRICS_CASE
    g = np.load(golden_dir / f"{case['name']}.npz")
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    dv, _ = core.danse(sc, dp)
    sig = core.generate_signals_for_snr_computation(dp, dv, sc, core.danse)
    ov = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive)
    osig = O.generate_signals_for_snr_computation(sc, dp, ov, vadMinProp=wp.vadMinProportionActive)
    ref, s0 = dp.referenceSensor, case['startIdx']
    worst = {}
    for k in range(len(case['M'])):
        nd = sc.wasn[k]
        m = DM.get_metrics(clean=nd.cleanspeech[:, ref], noiseOnly=nd.cleannoise[:, ref], noisy=nd.data[:, ref],
                           filtSpeech=sig['s'][:, k], filtNoise=sig['n'][:, k],
                           filtSpeech_c=sig['s_c'][:, k], filtNoise_c=sig['n_c'][:, k],
                           filtSpeech_l=sig['s_l'][:, k], filtNoise_l=sig['n_l'][:, k],
                           enhan=dv.d[:, k], enhan_c=dv.dCentr[:, k], enhan_l=dv.dLocal[:, k],
                           startIdx=s0, endIdx=nd.data.shape[0], fs=nd.fs, vad=nd.vad,
                           metricsToPlot=['snr', 'fwSNRseg', 'stoi'])
        for key in ('snr', 'fwSNRseg'):
            for fld in ('before', 'after', 'diff', 'afterCentr', 'afterLocal'):
                e = abs(getattr(m[key], fld) - float(g[f'{key}_{fld}_{k}']))
                worst[key] = max(worst.get(key, 0.0), e)
                assert e <= 0.01, (k, key, fld, e)
        cl = nd.cleanspeech[s0:, ref]
        for fld, est in (('after', ov.d[:, k]), ('afterCentr', ov.dCentr[:, k]), ('afterLocal', ov.dLocal[:, k]),
                         ('before', nd.data[:, ref])):
            e = abs(getattr(m['stoi'], fld) - MR.stoi(cl, est[s0:], nd.fs, extended=True))
            worst['stoi'] = max(worst.get('stoi', 0.0), e)
            assert e <= 0.01, (k, 'stoi', fld, e)
    print('worst |device - reference|:', worst, 'dSNR node 0', m['snr'].diff if k == 0 else None)
