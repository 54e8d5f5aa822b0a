"""Reference-API drivers (``danse_toolbox/d_core.py``) on the MI355X engine.

``danse(wasnObj, p)`` is the drop-in for the reference's
``danse_function`` (``d_core.py:26-102``): same arguments (a WASN whose nodes
carry ``data``/``timeStamps``/``fs``/``vadPerFrame``/``neighborsIdx`` and a
``DANSEparameters``), same returned fields.  ``danse_multi`` runs S
same-shape scenes in one batched engine (the Monte-Carlo battery use).
"""
from __future__ import annotations

import copy
import time

import numpy as np

from .engine import DanseEngine, beta_from_t50p
from .outputs import DANSEoutputs
from .params import PreComputedFilters


def prep_for_danse(p, wasnObj):
    """``d_core.prep_for_danse`` (``d_core.py:466-547``): forgetting factors
    per node and frame VAD."""
    for node in wasnObj.wasn:
        node.beta = (beta_from_t50p(p.danseParams.t_expAvg50p, node.fs, p.danseParams.Ns)
                     if p.danseParams.forcedBeta is None else p.danseParams.forcedBeta)
        node.betaWext = (beta_from_t50p(p.danseParams.t_expAvg50pExternalFilters, node.fs, p.danseParams.Ns)
                         if p.danseParams.forcedBetaExternalFilters is None else p.danseParams.forcedBetaExternalFilters)
    wasnObj.get_vad_per_frame(frameLen=p.danseParams.DFTsize, frameShift=p.danseParams.Ns,
                              minProportionActive=p.wasnParams.vadMinProportionActive)
    return p, wasnObj


def danse_multi(scenes, p, device=0, graph=True, keepHistory=True, yin='data', pregiven=None, smallDGrid=False,
                resident=False):
    """Run the online engine on S same-shape scenes at once; returns one
    output object per scene.  smallDGrid: the latency layout (GEVD filter
    dimensions <= 12 on the 4 x 4 lane-grid solver, DanseEngine); resident:
    the whole run in one persistent launch (csrc/resident.hpp)."""
    eng = DanseEngine(scenes, p, device=device, keepHistory=keepHistory, yin=yin, pregiven=pregiven,
                      smallDGrid=smallDGrid, resident=resident)
    try:
        eng.run(graph=graph)
        return eng.outputs()
    finally:
        eng.close()


def danse(wasnObj, p, device=0, graph=True):
    """``d_core.danse``: online fully connected DANSE of one WASN."""
    t0 = time.perf_counter()
    pg = p.preGivenFilters
    yin = 'data'
    pregiven = None
    if pg.active:
        yin = 'cleannoise' if pg.purpose == 'noise-only' else 'cleanspeech'
        pregiven = pg
    dv = danse_multi([wasnObj], p, device=device, graph=graph, yin=yin, pregiven=pregiven)[0]
    dv.wallSeconds = time.perf_counter() - t0
    return dv, wasnObj


def _family_batch(scenes, p, obs, device=0, yin='data', wGiven=None):
    """One ``obs='local'`` / ``'centr'`` batch engine run (one filter update
    per node, untrimmed MMSE cost); per-scene ``family_outputs``."""
    from .batch import BatchEngine
    eng = BatchEngine(scenes, p, device=device, costTrim=0, obs=obs, yin=yin, wGiven=wGiven)
    try:
        eng.run()
        return eng.family_outputs()
    finally:
        eng.close()


def danse_batch_multi(scenes, p, device=0):
    """Batch DANSE on S same-shape scenes at once (device batch engine).
    With ``computeCentralised`` / ``computeLocal`` the centralised and local
    batch estimates come first, as in ``d_core.danse_batch``
    (``d_core.py:282-283``, ``get_centralized_and_local_estimates``,
    ``d_batch.py:20-88``)."""
    from .batch import BatchEngine
    fam = {}
    for name, on in (('Centr', p.computeCentralised), ('Local', p.computeLocal)):
        if on:
            fam[name] = _family_batch(scenes, p, 'centr' if name == 'Centr' else 'local', device=device)
    eng = BatchEngine(scenes, p, device=device)
    try:
        eng.run()
        res = eng.outputs()
    finally:
        eng.close()
    for s, r in enumerate(res):
        for name, outs in fam.items():
            o = outs[s]
            suf = name[0].lower()
            setattr(r, f'w{name}', o.w)
            setattr(r, f'd{name}', o.d)
            setattr(r, f'dHat{name}', o.dhat)
            setattr(r, f'mmseCost{name}', o.mmseCost)
            # DANSEoutputs names (d_post.py:41-133)
            setattr(r, f'filters{name}', o.w)
            setattr(r, f'TDdesiredSignals_est_{suf}', o.d)
            setattr(r, f'STFTDdesiredSignals_est_{suf}', o.dhat)
    return res


def danse_batch(wasnObj, p, device=0):
    """``d_core.danse_batch`` (``d_core.py:251-352``): batch-mode fully
    connected DANSE of one WASN; returns ``(out, wasnObj)`` with the
    reference's output names (``filters``, ``TDdesiredSignals_est``,
    ``mmseCost``, ``wTilde``, ``wTildeExt``, ``d``, ``dhat``)."""
    t0 = time.perf_counter()
    out = danse_batch_multi([wasnObj], p, device=device)[0]
    out.wallSeconds = time.perf_counter() - t0
    return out, wasnObj


class BestPerf:
    """``get_best_perf``'s result (a ``BatchDANSEvariables`` in the
    reference): the fields ``include_best_perf_data`` and the SNR replays
    read (``d_post.py:152-182``)."""
    pass


def get_best_perf(wasnObj, p, wCentr=None, device=0):
    """``d_core.get_best_perf`` (``d_core.py:602-627``) for fully connected
    WASNs: centralised batch estimates without SROs
    (``init_from_wasn_for_best_perf``, ``d_classes.py:378-470``;
    ``get_centralized_estimates``, ``d_batch.py:90-125``) on the device batch
    engine (``obs='centr'``).  The scene generator applies no resampling, so
    the noSRO signals are the scene signals.  With ``p.preGivenFilters``
    active the noise-only / speech-only signals are filtered with slot 1 of
    ``wCentr``."""
    pg = p.preGivenFilters
    yin = 'data'
    if pg.active:
        yin = 'cleannoise' if pg.purpose == 'noise-only' else 'cleanspeech'
    o = _family_batch([wasnObj], p, 'centr', device=device, yin=yin, wGiven=wCentr)[0]
    bp = BestPerf()
    bp.wCentr, bp.dCentr, bp.dHatCentr, bp.mmseCostCentr = o.w, o.d, o.dhat, o.mmseCost
    bp.nNodes = wasnObj.nNodes
    bp.referenceSensor = p.referenceSensor
    bp.baseFs = wasnObj.wasn[p.referenceSensor].fs if hasattr(wasnObj, 'wasn') else None
    bp.cleanSpeechSignalsAtNodes = [nd.cleanspeech for nd in wasnObj.wasn]
    bp.cleanNoiseSignalsAtNodes = [nd.cleannoise for nd in wasnObj.wasn]
    return bp


def generate_signals_for_snr_computation(pD, dv, wasnObj, danse_function=danse, bestPerfRef=False, wCentrBatch=None):
    """``d_core.generate_signals_for_snr_computation`` (``d_core.py:550-599``):
    noise-only and speech-only replays with the recorded filters, and with
    ``bestPerfRef`` the same replays of the best-performance reference
    (``get_best_perf`` with ``wCentrBatch``)."""
    pU = copy.deepcopy(pD)
    pU.preGivenFilters = PreComputedFilters(
        active=True, internalFilters=dv.wTilde, externalFilters=dv.wTildeExt,
        filtersCentr=getattr(dv, 'wCentr', []), filtersSSBC=getattr(dv, 'wSSBC', []),
        filtersLocal=getattr(dv, 'wLocal', []), purpose='noise-only')
    dv_n, _ = danse_function(wasnObj, pU)
    bp_n = get_best_perf(wasnObj, pU, wCentr=wCentrBatch) if bestPerfRef else None
    pU.preGivenFilters.purpose = 'speech-only'
    dv_s, _ = danse_function(wasnObj, pU)
    bp_s = get_best_perf(wasnObj, pU, wCentr=wCentrBatch) if bestPerfRef else None
    out = {}
    for key, src in (('n', dv_n), ('s', dv_s)):
        out[key] = src.d
        out[f'{key}_c'] = getattr(src, 'dCentr', None)
        out[f'{key}_l'] = getattr(src, 'dLocal', None)
        out[f'{key}_ssbc'] = getattr(src, 'dSSBC', None)
    if bestPerfRef:
        out['n_bp'] = bp_n.dCentr
        out['s_bp'] = bp_s.dCentr
    return out


def format_output(p, dv, wasnObj, sigsSnr=None):
    """``d_core.format_output`` (``d_core.py:105-127``): the reference's
    ``DANSEoutputs`` from ``dv`` (and the SNR replay signals), and the
    enhanced signals written back into the WASN nodes."""
    out = DANSEoutputs()
    out.import_params(p)
    out.from_variables(dv)
    if sigsSnr is not None:
        out.from_snr_signals(sigsSnr)
    for k in range(len(wasnObj.wasn)):
        wasnObj.wasn[k].enhancedData = dv.d[:, k]
        if dv.computeCentralised:
            wasnObj.wasn[k].enhancedData_c = dv.dCentr[:, k]
        if dv.computeLocal:
            wasnObj.wasn[k].enhancedData_l = dv.dLocal[:, k]
        if dv.computeSingleSensorBroadcast:
            wasnObj.wasn[k].enhancedData_ssbc = dv.dSSBC[:, k]
    return out, wasnObj
