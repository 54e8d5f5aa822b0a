"""``tests/sandbox.py`` (``main`` / ``danse_it_up``, lines 14-160) on the
MI355X engine.

Same call shape and control flow as the reference: load the YAML (or take a
``TestParameters``), build the WASN, ``prep_for_danse``, run the danse
function selected by ``danse_it_up``, the noise-only / speech-only SNR
replays, and ``format_output``.  Differences, all loud:

* the WASN comes from the seeded random-IR scene generator
  (``danse_amd.scene.make_scene``); room acoustics and wav-file signals
  (``trueRoom``, ``signalType='from_file'``) raise NotImplementedError;
* ``postprocess`` (metrics, plots, exports; ``sandbox.py:162-``) is out of
  scope: ``main`` returns the formatted ``DANSEoutputs``;
* TI-DANSE (ad-hoc topologies) raises NotImplementedError, as the reference
  does for batch DANSE in ``danse_it_up``.
"""
from __future__ import annotations

import numpy as np

from . import core
from .params import TestParameters
from .scene import make_scene


def build_wasn(wasnParams, seed=None):
    """The random-IR stand-in for ``sig_ut.build_scenario`` +
    ``sig_ut.build_wasn`` (``sandbox.py:51-70``)."""
    wp = wasnParams
    if wp.trueRoom:
        raise NotImplementedError('trueRoom (pyroomacoustics room simulation) is out of scope: set '
                                  'wasnParams.trueRoom = False for the random-IR scene')
    if wp.signalType != 'random':
        raise NotImplementedError(f'signalType={wp.signalType!r}: only random signals (no wav files offline)')
    if wp.topologyParams.topologyType != 'fully-connected':
        raise NotImplementedError('ad-hoc topologies (TI-DANSE) are out of scope')
    rsp = wp.randSignalsParams
    return make_scene(list(np.asarray(wp.nSensorPerNode, dtype=int)), sigDur=wp.sigDur, fs=wp.fs,
                      seed=wp.generateRandomWASNwithSeed if seed is None else seed, snr=wp.snr,
                      selfnoiseSNR=wp.selfnoiseSNR, irDuration=wp.randIRsParams.duration,
                      pauseDuration=rsp.pauseDuration, pauseSpacing=rsp.pauseSpacing,
                      vadEnergyDecrease_dB=wp.VADenergyDecrease_dB, vadWinLength=wp.VADwinLength,
                      SROperNode=wp.SROperNode)


def main(p: TestParameters = None, cfgFilename: str = '', seed=None):
    """``sandbox.main`` (``sandbox.py:14-100``)."""
    if p is None:
        if not cfgFilename:
            raise ValueError('no parameters and no config file (the reference default, config_files/'
                             'sandbox_config.yaml, is not shipped here)')
        p = TestParameters().load_from_yaml(cfgFilename)
        p.danseParams.get_wasn_info(p.wasnParams)
    elif not getattr(p.danseParams, 'wasnInfoInitiated', False):
        p.danseParams.get_wasn_info(p.wasnParams)
    if not p.exportParams.check_export_folder():
        return None
    wasnObj = build_wasn(p.wasnParams, seed)
    p.danseParams.get_wasn_info(p.wasnParams)
    p, wasnObj = core.prep_for_danse(p, wasnObj)
    out, _ = danse_it_up(wasnObj, p)
    return out


def danse_it_up(wasnObj, p: TestParameters):
    """``sandbox.danse_it_up`` (``sandbox.py:102-160``)."""
    args = (wasnObj, p.danseParams)
    if not p.is_fully_connected_wasn():
        raise NotImplementedError('TI-DANSE (ad-hoc topologies) is out of scope')
    if p.danseParams.simType == 'batch':
        # the reference raises here too (sandbox.py:116-117); core.danse_batch
        # runs batch mode directly
        raise NotImplementedError('Batch mode not implemented / tested yet.')
    danse_function = core.danse
    dv, wasnObj = danse_function(*args)
    bp = p.exportParams.bestPerfReference
    # best possible performance (centralised, no SROs, batch), sandbox.py:132-155
    outBP = core.get_best_perf(*args) if bp else None
    sigsSnr = core.generate_signals_for_snr_computation(p.danseParams, dv, wasnObj, danse_function, bp,
                                                        wCentrBatch=outBP.wCentr if bp else None)
    out, wasnObj = core.format_output(p.danseParams, dv, wasnObj, sigsSnr=sigsSnr)
    if bp:
        out.include_best_perf_data(outBP, sigsSnr)
    return out, wasnObj
