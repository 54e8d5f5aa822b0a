"""Import harness for the reference Python toolbox (p-didier/danse) — THIS
CONTAINER ONLY.  Used exclusively by ``tests/golden/make_golden.py`` to
generate golden vectors; nothing on the GPU box imports it (the reference is
not present there).

Recipe:
* ``danse_toolbox/d_sros.py:8-13`` walks up the path until a directory named
  ``sounds-phd``; we import through a symlink ``<tmp>/sounds-phd/danse ->
  /root/reference`` so the walk terminates.
* Modules absent offline are stubbed: ``numba`` (jit/njit -> identity, the two
  jitted helpers are ``np.flip(np.argsort(.))`` and ``np.trace``),
  ``pyinstrument`` (no-op profiler), ``pesq``/``resampy``/``librosa``/
  ``pyroomacoustics``/``pyANFgen``/``dataclass_wizard``/``paderwasn``
  (import-time only; any call raises).  None of these take part in the
  arithmetic of the online/batch DANSE path.
* ``np.real_if_close`` -> ``np.real`` inside ``d_base`` only
  (SURVEY §8c shim 4: the reference otherwise crashes on a complex->float cast
  once |x| exceeds ~100; real parts are identical whenever it does not crash).
* ``scipy.signal.blackman`` alias for ``dxcpphat/sro_estimation.py:233``.
"""
from __future__ import annotations

import os
import sys
import types
import tempfile
from pathlib import Path

import numpy as np

REF = Path('/root/reference')
_loaded = None


def _stub(name: str, **attrs):
    mod = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(mod, k, v)
    sys.modules[name] = mod
    return mod


def _raise(*a, **k):
    raise RuntimeError('stubbed third-party function called (not available offline)')


def load():
    """Import the reference modules; returns a namespace with them."""
    global _loaded
    if _loaded is not None:
        return _loaded
    if not REF.is_dir():
        raise RuntimeError('/root/reference not present: golden generation only runs in the build container')
    os.environ['PYTHONDONTWRITEBYTECODE'] = '1'
    sys.dont_write_bytecode = True
    import matplotlib
    matplotlib.use('Agg')
    import scipy.signal
    import scipy.signal.windows
    if not hasattr(scipy.signal, 'blackman'):
        scipy.signal.blackman = scipy.signal.windows.blackman

    root = Path(tempfile.gettempdir()) / 'danse_refharness'
    sp = root / 'sounds-phd'
    (sp / '_third_parties').mkdir(parents=True, exist_ok=True)
    link = sp / 'danse'
    if not link.exists():
        link.symlink_to(REF)

    def identity_decorator(*a, **k):
        if len(a) == 1 and callable(a[0]) and not k:
            return a[0]
        return lambda f: f

    class _Profiler:
        def start(self): pass
        def stop(self): pass
        def print(self): pass

    _stub('numba', jit=identity_decorator, njit=identity_decorator)
    _stub('pyinstrument', Profiler=_Profiler)
    _stub('pesq', pesq=_raise)
    _stub('resampy', resample=_raise, core=types.SimpleNamespace(resample=_raise))
    _stub('librosa', load=_raise)
    pra = _stub('pyroomacoustics')
    pra.room = _stub('pyroomacoustics.room', ShoeBox=object)
    _stub('pyANFgen')
    _stub('pyANFgen.pyanfgen')
    _stub('pyANFgen.pyanfgen.utils', pyanfgen=_raise, ANFgenConfig=object)
    _stub('dataclass_wizard', fromdict=_raise, asdict=_raise)
    _stub('paderwasn')
    _stub('paderwasn.synchronization')
    _stub('paderwasn.synchronization.time_shift_estimation', max_time_lag_search=_raise)

    sys.path.insert(0, str(link))
    import danse_toolbox.d_base as base
    import danse_toolbox.d_classes as cl
    import danse_toolbox.d_core as core
    import danse_toolbox.d_batch as dbatch
    import siggen.classes as sgc
    # d_base only: route `np.real_if_close` to `np.real` through a proxy module
    # (d_classes' covariance gate keeps the true `np.real_if_close`).
    class _NpProxy(types.ModuleType):
        def __getattr__(self, name):
            return getattr(np, name)
    proxy = _NpProxy('numpy')
    proxy.real_if_close = np.real
    base.np = proxy
    ns = types.SimpleNamespace(base=base, cl=cl, core=core, dbatch=dbatch, sgc=sgc)
    _loaded = ns
    return ns


def to_ref_wasn(ns, scene):
    """Inject our scene arrays into reference ``Node``/``WASN`` objects."""
    wasn = []
    for node in scene.wasn:
        wasn.append(ns.sgc.Node(
            index=node.index,
            nSensors=node.nSensors,
            refSensorIdx=0,
            sro=node.sro,
            fs=node.fs,
            data=node.data.copy(),
            data_noSRO=node.data.copy(),
            cleanspeech=node.cleanspeech.copy(),
            cleanspeech_noSRO=node.cleanspeech.copy(),
            cleannoise=node.cleannoise.copy(),
            cleannoise_noSRO=node.cleannoise.copy(),
            timeStamps=node.timeStamps.copy(),
            neighborsIdx=list(node.neighborsIdx),
            vad=node.vad.copy(),
        ))
    w = ns.sgc.WASN(wasn=wasn, adjacencyMatrix=np.array([]))
    return w


def make_params(ns, nSensorPerNode, fs=16000.0, **danse_overrides):
    """Reference ``TestParameters`` for a fully connected random-IR scene."""
    p = ns.cl.TestParameters()
    # Fresh sub-dataclass instances (class-level defaults are shared/mutated by load_from_yaml).
    p.wasnParams = ns.sgc.WASNparameters(
        trueRoom=False, signalType='random', fs=fs,
        nSensorPerNode=list(nSensorPerNode),
        SROperNode=np.zeros(len(nSensorPerNode)),
        topologyParams=ns.sgc.TopologyParameters(topologyType='fully-connected', seed=12348),
    )
    p.danseParams = ns.base.DANSEparameters(
        printoutsAndPlotting=ns.base.PrintoutsAndPlotting(verbose=False, printout_profiler=False,
                                                         printout_eventsParser=False,
                                                         printout_externalFilterUpdate=False),
        cohDrift=ns.base.CohDriftParameters(),
        preGivenFilters=ns.base.PreComputedFilters(),
    )
    for k, v in danse_overrides.items():
        if not hasattr(p.danseParams, k):
            raise KeyError(k)
        if k == 'cohDrift' and isinstance(v, dict):
            v = ns.base.CohDriftParameters(**v)
        setattr(p.danseParams, k, v)
    p.danseParams.__post_init__()
    p.exportParams = ns.cl.ExportParameters(bypassAllExports=True, conditionNumberPlot=False)
    p.__post_init__()
    p.danseParams.get_wasn_info(p.wasnParams)
    return p


def prep(ns, p, refWasn):
    return ns.core.prep_for_danse(p, refWasn)
