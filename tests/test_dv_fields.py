"""The reference's ``dv`` output surface, on CPU:

* every attribute ``DANSEoutputs.from_variables`` / ``format_output`` read
  (``d_post.py:41-133``, ``d_core.py:105-127``; the list is parsed from the
  reference source into the ``fields_*`` fixtures) is produced by the
  engine's outputs, or is one of the named exceptions;
* the schedule-derived fields (SRO estimates / residuals, flag iterations,
  first-update instant, MSE-cost arrays) equal the reference's on the
  ``fields_*`` fixtures (``danse_amd.outputs.host_fields``);
* ``DANSEoutputs`` / ``format_output`` map the fields like the reference.
The device-computed ``yinSTFT`` is checked in ``test_gpu_engine_modes.py``.
"""
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest

from golden_cases import ONLINE_CASES, FIELD_CASES
from _util import make_case_params, make_case_scene

from danse_amd import outputs as OUT
from danse_amd.scheduler import initialize_events, compile_rounds, compile_rounds_fs
from danse_amd.outputs import stft_frames

GOLD = Path(__file__).parent / 'golden'

# read by from_variables only outside this path: batch mode (mmseCost*),
# TI-DANSE (etaMkFullTD, under hasattr), saveConditionNumber (condNumbers,
# set to None with a warning)
EXCEPTIONS = {'mmseCost', 'mmseCostInit', 'mmseCostLocal', 'mmseCostCentr', 'etaMkFullTD', 'condNumbers'}


def _case(name):
    return next(c for c in ONLINE_CASES if c['name'] == name)


def test_dv_field_set_covers_reference():
    z = np.load(GOLD / f'fields_{FIELD_CASES[0]}.npz')
    read = set(str(x) for x in z['dvFieldsRead'])
    produced = set(OUT.ONLINE_DV_FIELDS)
    for v in OUT.FAMILY_DV_FIELDS.values():
        produced |= set(v)
    missing = read - produced - EXCEPTIONS
    assert not missing, missing
    # the engine's output assembly sets every one of them (source check: no GPU here)
    src = (Path(OUT.__file__).parent / 'engine.py').read_text() + Path(OUT.__file__).read_text()
    for nm in sorted(read - EXCEPTIONS):
        assert f"'{nm}'" in src or f'.{nm} =' in src or f"r.{nm}" in src, nm


@pytest.mark.parametrize('name', FIELD_CASES)
def test_host_fields_match_reference(name):
    case = _case(name)
    z = np.load(GOLD / f'fields_{name}.npz')
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    K = len(case['M'])
    neighbors = [list(n.neighborsIdx) for n in sc.wasn]
    events, fs = initialize_events([n.timeStamps for n in sc.wasn], [n.fs for n in sc.wasn], dp, neighbors)
    if dp.broadcastType == 'fewSamples':
        rt = compile_rounds_fs(events, fs, dp, K, [n.timeStamps for n in sc.wasn], [n.nSensors for n in sc.wasn])
    else:
        rt = compile_rounds(events, fs, dp, K)
    T = sc.wasn[0].data.shape[0]
    nIter = int((T - dp.DFTsize) / dp.Ns) + 1
    # first DANSE solve round of node p.referenceSensor: gate from the counters, then the schedule
    kr = dp.referenceSensor
    D = sc.wasn[kr].nSensors + K - 1
    v = sc.wasn[kr].vadPerFrame[:rt.nRounds]
    ny = np.cumsum(v)
    nn = np.arange(1, len(v) + 1) - ny
    gate = np.maximum.accumulate((ny > D) & (nn > D) & (rt.t[:, kr] >= dp.startUpdatesAfterAtLeast))
    solve = gate & (rt.doSolve[:, kr] != 0)
    fsr = int(np.argmax(solve)) if solve.any() else -1
    nseg = stft_frames(T, dp.DFTsize, dp.Ns)
    f = OUT.host_fields(dp, [n.sro for n in sc.wasn], neighbors, rt, nIter, nseg, fsr)
    cohDrift = case['danse'].get('estimateSROs') == 'CohDrift'
    if cohDrift:
        # data-driven estimates (the device's, danse_engine_sro_estimates): the
        # float64 oracle's estimator against the reference's own values here,
        # the device against the oracle in test_gpu_engine_modes.py
        from oracle import danse_ref_cpu as O
        ov = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive).run()
    for k in range(K):
        if cohDrift:
            for nm in ('SROsResiduals', 'SROsEstimates'):
                ref = z[f'{nm}_{k}']
                got = np.asarray(getattr(ov, nm)[k])[:ref.shape[0]]
                np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-15 * max(1.0, np.max(np.abs(ref))))
        else:
            np.testing.assert_allclose(f['SROsResiduals'][k], z[f'SROsResiduals_{k}'], rtol=0, atol=1e-18)
            np.testing.assert_allclose(f['SROsEstimates'][k], z[f'SROsEstimates_{k}'], rtol=0, atol=1e-18)
        assert list(f['flagIterations'][k]) == list(z[f'flagIterations_{k}']), k
    ref_first = float(z['firstDANSEupdateRefSensor'])
    assert f['firstDANSEupdateRefSensor'] == pytest.approx(ref_first, abs=1e-12)
    for nm in ('mseCostOnline', 'mseCostOnline_c', 'mseCostOnline_l'):
        assert list(f[nm].shape) == list(z[f'{nm}_shape'])
        assert all(x is None for x in np.ravel(f[nm])) == bool(z[f'{nm}_allNone'])
    assert nseg == int(z['yCentrBatch_shape'][1])


def test_format_output_mapping():
    from danse_amd import core
    from danse_amd.params import DANSEparameters
    p = DANSEparameters(simType='online', computeLocal=True)
    p.__post_init__()
    K, T = 2, 100
    dv = SimpleNamespace(**{nm: nm for nm in OUT.ONLINE_DV_FIELDS})
    dv.d = np.zeros((T, K))
    dv.dLocal = np.ones((T, K))
    for nm in ('dHatLocal', 'wLocal', 'mseCostOnline_l'):
        setattr(dv, nm, nm)
    dv.computeCentralised, dv.computeLocal, dv.computeSingleSensorBroadcast = False, True, False
    wasn = SimpleNamespace(wasn=[SimpleNamespace() for _ in range(K)])
    sigs = {k: k for k in ('s', 'n', 's_c', 'n_c', 's_l', 'n_l', 's_ssbc', 'n_ssbc')}
    out, wasn = core.format_output(p, dv, wasn, sigsSnr=sigs)
    assert out.initialised and out.simType == 'online'
    assert out.TDdesiredSignals_est is dv.d and out.TDdesiredSignals_est_l is dv.dLocal
    assert out.TDdesiredSignals_est_c is None and out.filtersCentr is None
    assert out.filters == 'wTilde' and out.filtersEXT == 'wTildeExt' and out.yinSTFT == 'yinSTFT'
    assert out.firstUpRefSensor == 'firstDANSEupdateRefSensor' and out.SROgroundTruth == 'SROsppm'
    assert out.mseCostOnline_l == 'mseCostOnline_l' and out.filtersLocal == 'wLocal'
    assert out.TDfiltSpeech == 's' and out.TDfiltNoise_ssbc == 'n_ssbc'
    assert np.array_equal(wasn.wasn[1].enhancedData, dv.d[:, 1])
    assert np.array_equal(wasn.wasn[0].enhancedData_l, dv.dLocal[:, 0])


def test_sandbox_mirror_errors():
    """danse_it_up raises where the reference does (batch mode) and where the
    device path stops (TI-DANSE, bestPerfReference, room acoustics)."""
    from danse_amd import sandbox, params as P
    tp = P.TestParameters(wasnParams=P.WASNparameters(trueRoom=False, signalType='random', nSensorPerNode=[1, 1]))
    with pytest.raises(NotImplementedError):
        sandbox.danse_it_up(None, tp)      # bestPerfReference defaults to True
    tp.danseParams.simType = 'batch'
    with pytest.raises(NotImplementedError, match='Batch mode'):
        sandbox.danse_it_up(None, tp)
    wp = P.WASNparameters(trueRoom=True, nSensorPerNode=[1, 1])
    with pytest.raises(NotImplementedError):
        sandbox.build_wasn(wp)


def test_outputs_disk_format(tmp_path):
    """DANSEoutputs.save / load / save_metrics (d_post.py:184-212,
    dataclass_methods.py:13-117): <folder>/DANSEoutputs.pkl.gz, the text view
    and metrics.pkl; 'json' raises as in the reference; load round-trips."""
    import gzip
    import pickle
    from danse_amd.params import DANSEparameters
    p = DANSEparameters(simType='online')
    p.__post_init__()
    out = OUT.DANSEoutputs().import_params(p)
    assert isinstance(out.check_init(), ValueError)
    out.TDdesiredSignals_est = np.arange(12.0).reshape(6, 2)
    out.filters = [np.ones((3, 4, 2), dtype=np.complex64)]
    out.metrics = {'snr': {'Node1': 1.5}}
    out.initialised = True
    d = tmp_path / 'res'
    out.save(str(d), light=True)
    assert (d / 'DANSEoutputs.pkl.gz').is_file() and (d / 'DANSEoutputs_text.txt').is_file()
    txt = (d / 'DANSEoutputs_text.txt').read_text()
    assert txt.startswith('>--------DANSEoutputs class instance') and ' - simType = online' in txt
    back = OUT.DANSEoutputs().load(str(d))
    assert np.array_equal(back.TDdesiredSignals_est, out.TDdesiredSignals_est)
    assert back.filters[0].dtype == np.complex64 and back.simType == 'online'
    # (light: the reference saves the full object anyway)
    assert hasattr(back, 'TDdesiredSignals_est')
    out.save_metrics(str(d))
    with open(d / 'metrics.pkl', 'rb') as f:
        assert pickle.load(f) == out.metrics
    with gzip.open(d / 'DANSEoutputs.pkl.gz', 'rb') as f:
        assert type(pickle.load(f)).__name__ == 'DANSEoutputs'
    with pytest.raises(ValueError, match='NOT YET'):
        out.save(str(tmp_path / 'j'), exportType='json')
    with pytest.raises(ValueError):
        OUT.DANSEoutputs().load(str(tmp_path / 'missing'))
