"""Generate golden vectors by running the REFERENCE (p-didier/danse, imported
through ``_refharness``) on seeded synthetic scenes.  Build-container only
(needs /root/reference); the committed ``.npz`` files are the only thing that
travels.  Inputs are not stored: they are regenerated from the seed by
``danse_amd.scene.make_scene`` and pinned by a sha256 digest stored in each
fixture.

Usage:  python tests/golden/make_golden.py            (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(HERE))

import _refharness as H  # noqa: E402
from danse_amd.scene import make_scene, scene_digest  # noqa: E402
from golden_cases import ONLINE_CASES, BATCH_CASES, SRO_EVENT_CASES, KAT_CASES, kat_inputs, BESTPERF_CASES  # noqa: E402
from golden_cases import DXCP_CASES, dxcp_inputs, TZ_CASES, tz_inputs, CLDXCP_CASES, cldxcp_acs  # noqa: E402
from golden_cases import METRIC_CASES, metric_inputs, GETMETRICS_CASE, get_metrics_inputs  # noqa: E402
from golden_cases import FIELD_CASES, FIELD_STFT_BIN_STEP, STOI_CASES, stoi_inputs, E2E_METRICS_CASE  # noqa: E402
from golden_cases import SCENE_CASES, scene_inputs, COND_CASES, REF_MODES_CASE  # noqa: E402


def _run_online(ns, case):
    sros = case.get('sros')
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'], SROperNode=sros)
    p = H.make_params(ns, case['M'], **case['danse'])
    if sros is not None:
        p.wasnParams.SROperNode = np.array(sros, dtype=float)
    w = H.to_ref_wasn(ns, sc)
    p, w = H.prep(ns, p, w)
    t0 = time.time()
    dv, w = ns.core.danse(w, p.danseParams)
    el = time.time() - t0
    out = {'digest': scene_digest(sc), 'ref_seconds': el}
    K = len(case['M'])
    every = case.get('wEvery', 16)
    asy = 'seq' not in case['danse']['nodeUpdating']
    out['d'] = dv.d
    out['dhat'] = dv.dhat[:, ::every, :]
    for nm, fl in [('dLocal', 'computeLocal'), ('dCentr', 'computeCentralised'), ('dSSBC', 'computeSingleSensorBroadcast')]:
        if case['danse'].get(fl, False):
            out[nm] = getattr(dv, nm)
    for k in range(K):
        out[f'w_{k}'] = dv.wTilde[k][:, ::every, :]
        if asy:
            out[f'wExt_{k}'] = dv.wTildeExt[k][:, ::every, :]
        if k < 2:
            out[f'z_{k}'] = dv.zFullTD[k]
        if case['danse'].get('computeLocal', False):
            out[f'wLocal_{k}'] = dv.wLocal[k][:, ::every, :]
        if case['danse'].get('computeCentralised', False):
            out[f'wCentr_{k}'] = dv.wCentr[k][:, ::every, :]
    out['startUpdates'] = np.array(dv.startUpdates)
    out['nInternalFilterUps'] = np.array(dv.nInternalFilterUps)
    if case.get('snr_replay', False):
        sigs = ns.core.generate_signals_for_snr_computation(p.danseParams, dv, w, ns.core.danse)
        for key in ['n', 's']:
            out[f'snr_{key}'] = sigs[key]
    return out


def _dv_fields_read():
    """The dv attributes d_post.DANSEoutputs.from_variables and
    d_core.format_output read (parsed from the reference source)."""
    import ast
    names = set()
    for rel, fn in (('danse_toolbox/d_post.py', 'from_variables'), ('danse_toolbox/d_core.py', 'format_output')):
        tree = ast.parse((H.REF / rel).read_text())
        for node in ast.walk(tree):
            if isinstance(node, ast.FunctionDef) and node.name == fn:
                for sub in ast.walk(node):
                    if isinstance(sub, ast.Attribute) and isinstance(sub.value, ast.Name) and sub.value.id == 'dv':
                        names.add(sub.attr)
    return sorted(names)


def _run_fields(ns, name):
    case = next(c for c in ONLINE_CASES if c['name'] == name)
    sros = case.get('sros')
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'], SROperNode=sros)
    p = H.make_params(ns, case['M'], **case['danse'])
    if sros is not None:
        p.wasnParams.SROperNode = np.array(sros, dtype=float)
    w = H.to_ref_wasn(ns, sc)
    p, w = H.prep(ns, p, w)
    dv, w = ns.core.danse(w, p.danseParams)
    K = len(case['M'])
    out = {'digest': scene_digest(sc), 'dvFieldsRead': np.array(_dv_fields_read())}
    for k in range(K):
        out[f'SROsEstimates_{k}'] = np.asarray(dv.SROsEstimates[k])
        out[f'SROsResiduals_{k}'] = np.asarray(dv.SROsResiduals[k])
        out[f'flagIterations_{k}'] = np.asarray(dv.flagIterations[k], dtype=np.int64)
        out[f'yinSTFT_{k}'] = dv.yinSTFT[k][::FIELD_STFT_BIN_STEP]
    out['yCentrBatch_shape'] = np.array(dv.yCentrBatch.shape)
    f = dv.firstDANSEupdateRefSensor
    out['firstDANSEupdateRefSensor'] = np.array(np.nan if f is None else float(f))
    for nm in ('mseCostOnline', 'mseCostOnline_c', 'mseCostOnline_l'):
        m = getattr(dv, nm)
        out[f'{nm}_shape'] = np.array(m.shape)
        out[f'{nm}_allNone'] = np.array(all(x is None for x in np.ravel(m)))
    return out


def _run_batch(ns, case):
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'])
    p = H.make_params(ns, case['M'], **case['danse'])
    w = H.to_ref_wasn(ns, sc)
    p, w = H.prep(ns, p, w)
    t0 = time.time()
    out_, w = ns.core.danse_batch(w, p.danseParams)
    el = time.time() - t0
    out = {'digest': scene_digest(sc), 'ref_seconds': el, 'd': out_.TDdesiredSignals_est,
           'mmseCost': np.array(out_.mmseCost, dtype=float)}
    for k in range(len(case['M'])):
        out[f'w_{k}'] = out_.filters[k][:, :case['danse']['maxBatchUpdates'] + 1, :]
    if case['danse'].get('computeCentralised', False):
        out['dCentr'] = out_.TDdesiredSignals_est_c
        out['mmseCostCentr'] = np.array(out_.mmseCostCentr, dtype=float)
        for k in range(len(case['M'])):
            out[f'wCentr_{k}'] = out_.filtersCentr[k][:, :2, :]
    if case['danse'].get('computeLocal', False):
        out['dLocal'] = out_.TDdesiredSignals_est_l
        out['mmseCostLocal'] = np.array(out_.mmseCostLocal, dtype=float)
        for k in range(len(case['M'])):
            out[f'wLocal_{k}'] = out_.filtersLocal[k][:, :2, :]
    return out


def _run_best_perf(ns, case):
    import copy
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'])
    p = H.make_params(ns, case['M'], **case['danse'])
    w = H.to_ref_wasn(ns, sc)
    p, w = H.prep(ns, p, w)
    bp = ns.core.get_best_perf(w, p.danseParams)
    out = {'digest': scene_digest(sc), 'dCentr': bp.dCentr, 'mmseCostCentr': np.array(bp.mmseCostCentr, dtype=float)}
    for k in range(len(case['M'])):
        out[f'wCentr_{k}'] = bp.wCentr[k][:, :2, :]
    pU = copy.deepcopy(p.danseParams)
    for purpose in ('noise-only', 'speech-only'):
        pU.preGivenFilters = ns.base.PreComputedFilters(active=True, purpose=purpose)
        o = ns.core.get_best_perf(w, pU, wCentr=bp.wCentr)
        out[f'dCentr_{purpose[0]}'] = o.dCentr
    return out


def _run_sro_events(ns, case):
    sc = make_scene(case['M'], sigDur=case['dur'], seed=0, SROperNode=case['sros'])
    p = H.make_params(ns, case['M'], **case['danse'])
    # WASNparameters SROs so that prep/checks see them
    p.wasnParams.SROperNode = np.array(case['sros'], dtype=float)
    w = H.to_ref_wasn(ns, sc)
    ev, fs, _ = ns.base.initialize_events(
        np.stack([n.timeStamps for n in sc.wasn], axis=1), p.danseParams, w)
    rows = []
    for e in ev:
        for ii in range(e.nEvents):
            rows.append((e.t, int(e.nodes[ii]), 0 if e.type[ii] == 'bc' else 1, int(e.bypassUpdate[ii])))
    rows = np.array(rows, dtype=[('t', 'f8'), ('node', 'i4'), ('type', 'i4'), ('bypass', 'i4')])
    return {'events': rows, 'fs': fs, 'n_instants': len(ev)}


def _run_kat(ns, case):
    Ryy, Rnn = kat_inputs(case)
    fn = ns.cl.update_w_gevd if case['gevd'] else ns.cl.update_w
    w = fn(Ryy, Rnn, refSensorIdx=case['ref'], rank=case.get('rank', 1))
    return {'w': w}


def _run_dxcp(ns, case):
    import sro_estimation   # dxcpphat/, on sys.path once the reference is loaded (d_sros.py:12)
    x1, x2 = dxcp_inputs(case)
    est = sro_estimation.DXCPPhaT()
    n = len(x1) // 2048
    sro = np.zeros(n)
    sto = np.zeros(n)
    for i in range(n):
        fr = np.stack((x1[i * 2048:(i + 1) * 2048], x2[i * 2048:(i + 1) * 2048]), axis=1)
        out = est.process_data(fr)
        sro[i] = out['SROppm_est_out']
        sto[i] = out['STOsmp_est_out']
    return {'sro': sro, 'sto': sto}


def _run_cldxcp(ns, case):
    import sro_estimation   # dxcpphat/ (on sys.path once the reference is loaded)
    x1, x2 = dxcp_inputs(case)
    cl = sro_estimation.CL_DXCPPhaT(start_delay=case['startDelay'])
    n = len(x1) // 2048
    acs = cldxcp_acs(case, n)
    out = np.zeros((n, 3))
    zi = np.zeros((n, 2048))
    for i in range(n):
        fr = np.stack((x1[i * 2048:(i + 1) * 2048], x2[i * 2048:(i + 1) * 2048]), axis=1)
        d, s_, sh, z = cl.process(fr, int(acs[i]))
        out[i] = (d, s_, sh)
        zi[i] = z
    return {'out': out, 'zi': zi[::5]}


def _run_tz(ns, case):
    wHat, yq, h, f, wPrev = tz_inputs(case)
    z, wIR = ns.base.danse_compression_few_samples(yq, wHat, case['L'], wPrev, h, f, case['Ns'],
                                                   updateBroadcastFilter=case['update'])
    return {'z': z, 'wIR': wIR}


def _run_metrics(ns, case):
    import danse_toolbox.d_eval as ev   # importable once the reference is loaded
    clean, enh, s, n, vad = metric_inputs(case)
    kw = {k: case[k] for k in ('frameLen', 'overlap', 'gamma') if k in case}
    fw = ev.get_fwsnrseg(clean, enh, case['fs'], **kw)
    return {'fw': np.asarray(fw, dtype=np.float64), 'fwMean': np.mean(fw),
            'snr': np.asarray(ev.get_snr(s, n, vad)), 'snrAll': np.asarray(ev.get_snr(s, n, vad, bypassVADuse=True)),
            'snr1': np.asarray(ev.get_snr(s[:, 0], n[:, 0], vad[:, 0]))}


def _run_get_metrics(ns, case):
    import danse_toolbox.d_eval as ev
    m = ev.get_metrics(**get_metrics_inputs(case), fs=case['fs'], startIdx=case['startIdx'], endIdx=case['endIdx'],
                       metricsToPlot=['snr', 'fwSNRseg'])
    out = {}
    for key in ('snr', 'fwSNRseg'):
        for fld in ('before', 'after', 'diff', 'afterCentr', 'afterLocal'):
            out[f'{key}_{fld}'] = np.float64(getattr(m[key], fld))
    return out


def _run_stoi(ns, case):
    import importlib
    st = importlib.import_module('danse_toolbox.mypystoi.stoi')   # the module (the package re-exports a function of that name)
    x, y = stoi_inputs(case)
    fn = getattr(st, case['fn'])
    np.random.seed(0)   # row_col_normalize adds EPS-scaled noise from the global generator
    return {'estoi': np.float64(fn(x, y, case['fs'], extended=True)),
            'stoi': np.float64(fn(x, y, case['fs'], extended=False))}


def _run_e2e_metrics(ns, case):
    import danse_toolbox.d_eval as ev
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'])
    p = H.make_params(ns, case['M'], **case['danse'])
    w = H.to_ref_wasn(ns, sc)
    p, w = H.prep(ns, p, w)
    dv, w = ns.core.danse(w, p.danseParams)
    sigs = ns.core.generate_signals_for_snr_computation(p.danseParams, dv, w, ns.core.danse)
    ref = p.danseParams.referenceSensor
    out = {'digest': scene_digest(sc)}
    for k in range(len(case['M'])):
        nd = sc.wasn[k]
        m = ev.get_metrics(clean=nd.cleanspeech[:, ref], noiseOnly=nd.cleannoise[:, ref], noisy=nd.data[:, ref],
                           filtSpeech=sigs['s'][:, k], filtNoise=sigs['n'][:, k],
                           filtSpeech_c=sigs['s_c'][:, k], filtNoise_c=sigs['n_c'][:, k],
                           filtSpeech_l=sigs['s_l'][:, k], filtNoise_l=sigs['n_l'][:, k],
                           enhan=dv.d[:, k], enhan_c=dv.dCentr[:, k], enhan_l=dv.dLocal[:, k],
                           startIdx=case['startIdx'], endIdx=nd.data.shape[0], fs=nd.fs, vad=nd.vad,
                           metricsToPlot=['snr', 'fwSNRseg'])
        for key in ('snr', 'fwSNRseg'):
            for fld in ('before', 'after', 'diff', 'afterCentr', 'afterLocal'):
                out[f'{key}_{fld}_{k}'] = np.float64(getattr(m[key], fld))
    return out


def _run_scene(ns, case):
    """The reference's get_vad (siggen/utils.py:834-893) on injected inputs,
    and oracleVAD on the float32-rounded wet reference-sensor signals."""
    import tempfile
    import siggen.utils as sgu
    x, h = scene_inputs(case)
    M = case['M']
    p = ns.sgc.WASNparameters(trueRoom=False, signalType='random', fs=case['fs'], nSensorPerNode=list(M),
                              SROperNode=np.zeros(len(M)),
                              topologyParams=ns.sgc.TopologyParameters(topologyType='fully-connected', seed=12348))
    p.VADwinLength = case['vadWinLength']
    p.VADenergyDecrease_dB = case['vadEnergyDecrease_dB']
    p.VADenergyFactor = 10 ** (p.VADenergyDecrease_dB / 10)
    p.enableVADloadFromFile = False
    p.vadFilesFolder = tempfile.mkdtemp(prefix='danse_vad_')
    rirs, c = [], 0
    for m in M:
        rirs.append([[h[c + i]] for i in range(m)])
        c += m
    vad, wet = sgu.get_vad(rirs, x[:, None], p)
    wetAll = np.concatenate(wet, axis=0)                  # [sum M][T]
    ref = np.cumsum([0] + list(M))[:-1]
    vad32 = np.stack([sgu.oracleVAD(wetAll[b].astype(np.float32).astype(np.float64), tw=p.VADwinLength,
                                    thrs=np.amax(wetAll[b].astype(np.float32).astype(np.float64) ** 2) /
                                    p.VADenergyFactor, Fs=p.fs)[0] for b in ref])
    return {'x': x, 'h': h, 'wet': wetAll, 'vad': vad[:, :, 0].T.astype(np.uint8), 'vad32': vad32.astype(np.uint8)}


def _run_cond(ns, case):
    """dv.condNumbers of the reference's online run (DANSE and local Ryy)."""
    sc = make_scene(case['M'], sigDur=case['dur'], seed=case['seed'])
    p = H.make_params(ns, case['M'], **case['danse'])
    # (TestParameters.__post_init__ ties saveConditionNumber to
    # exportParams.conditionNumberPlot, d_classes.py:226-230)
    p.exportParams.conditionNumberPlot = True
    p.danseParams.saveConditionNumber = True
    w = H.to_ref_wasn(ns, sc)
    p, w = H.prep(ns, p, w)
    dv, w = ns.core.danse(w, p.danseParams)
    cn = dv.condNumbers
    out = {'digest': scene_digest(sc)}
    for k in range(len(case['M'])):
        for fam in ('DANSE', 'Local'):
            out[f'cn_{fam}_{k}'] = np.asarray(getattr(cn, f'cn_Ryy{fam}')[k])
            out[f'iter_{fam}_{k}'] = np.asarray(getattr(cn, f'iter_cn_Ryy{fam}')[k], dtype=np.int64)
    return out


def _run_modes(ns, case):
    """The reference's outcome (ran / the exception it raised) for the online
    modes whose error behaviour the device path mirrors."""
    out = {}
    for key, extra in case['modes'].items():
        sc = make_scene([2, 3], sigDur=2.0, seed=5)
        p = H.make_params(ns, [2, 3], **dict(case['base'], nodeUpdating='asy', **extra))
        w = H.to_ref_wasn(ns, sc)
        p, w = H.prep(ns, p, w)
        assert all(getattr(p.danseParams, a) == v for a, v in extra.items()), 'parameter not applied'
        try:
            ns.core.danse(w, p.danseParams)
            out[key] = np.array('ran')
        except Exception as e:   # noqa: BLE001 -- the outcome is what is recorded
            out[key] = np.array(f'{type(e).__name__}: {e}')
    return out


def main():
    ns = H.load()
    only = sys.argv[1:]
    jobs = [('online', c, _run_online) for c in ONLINE_CASES] + \
           [('batch', c, _run_batch) for c in BATCH_CASES] + \
           [('bestperf', c, _run_best_perf) for c in BESTPERF_CASES] + \
           [('events', c, _run_sro_events) for c in SRO_EVENT_CASES] + \
           [('kat', c, _run_kat) for c in KAT_CASES] + \
           [('dxcp', c, _run_dxcp) for c in DXCP_CASES] + \
           [('cldxcp', c, _run_cldxcp) for c in CLDXCP_CASES] + \
           [('tz', c, _run_tz) for c in TZ_CASES] + \
           [('metrics', c, _run_metrics) for c in METRIC_CASES] + \
           [('metrics', GETMETRICS_CASE, _run_get_metrics)] + \
           [('stoi', c, _run_stoi) for c in STOI_CASES] + \
           [('metrics', E2E_METRICS_CASE, _run_e2e_metrics)] + \
           [('scene', c, _run_scene) for c in SCENE_CASES] + \
           [('cond', c, _run_cond) for c in COND_CASES] + \
           [('fields', dict(name=f'fields_{c}', src=c), lambda ns, c: _run_fields(ns, c['src'])) for c in FIELD_CASES] + \
           [('modes', REF_MODES_CASE, _run_modes)]
    for kind, case, fn in jobs:
        name = case['name']
        if only and name not in only:
            continue
        t0 = time.time()
        out = fn(ns, case)
        np.savez_compressed(HERE / f'{name}.npz', **out)
        sz = os.path.getsize(HERE / f'{name}.npz') / 1e6
        print(f'{kind:7s} {name:28s} {time.time() - t0:7.1f}s  {sz:6.2f} MB', flush=True)


if __name__ == '__main__':
    main()
