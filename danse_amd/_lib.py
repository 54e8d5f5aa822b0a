"""ctypes binding of the C-ABI in ``include/danse_mi355x.h``.

The shared library ``libdanse_mi355x.so`` is built in-tree by
``danse_amd.build.build()`` (hipcc, gfx950).  There is no fallback: if the
library is missing or fails to load, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_NAME = 'libdanse_mi355x.so'
# (DANSE_LIB: an alternative build of the same library, for A/B timing of
# compile-time variants; the in-tree library otherwise)
LIB_PATH = Path(os.environ['DANSE_LIB']) if os.environ.get('DANSE_LIB') else Path(__file__).resolve().parent / LIB_NAME

_c_i32 = ctypes.c_int32
_p_i32 = ctypes.POINTER(ctypes.c_int32)
_p_f32 = ctypes.POINTER(ctypes.c_float)
_p_u8 = ctypes.POINTER(ctypes.c_uint8)

FAM_DANSE, FAM_LOCAL, FAM_CENTR, FAM_SSBC = 0, 1, 2, 3
OP_KEEP, OP_SET, OP_AVG = 0, 1, 2
FLAG_SOLVE = 0x10
FLAG_EXT_TARGET = 0x20
FLAG_PREGIVEN = 0x40
FLAG_INITSLOT = 0x80
EXT_COPY, EXT_RELAX, EXT_KEEP, EXT_REFONLY = 0, 1, 2, 3
OUT_W, OUT_WEXT, OUT_D, OUT_DHAT, OUT_Z, OUT_DIAG = 0, 1, 2, 3, 4, 5


class SceneCfg(ctypes.Structure):
    _fields_ = [
        ('S', _c_i32), ('K', _c_i32), ('M', _p_i32), ('T', _c_i32), ('nIR', _c_i32), ('seed', ctypes.c_int64),
        ('fs', ctypes.c_double), ('snr', ctypes.c_double), ('selfnoiseSNR', ctypes.c_double),
        ('pauseDuration', ctypes.c_double), ('pauseSpacing', ctypes.c_double),
        ('vadEnergyDecrease_dB', ctypes.c_double), ('vadWinLength', ctypes.c_double),
        ('sroPpm', ctypes.POINTER(ctypes.c_double)),
    ]


class DanseCfg(ctypes.Structure):
    _fields_ = [
        ('S', _c_i32), ('K', _c_i32), ('M', _p_i32),
        ('N', _c_i32), ('Ns', _c_i32), ('T', _c_i32), ('R', _c_i32),
        ('k0', _c_i32), ('k1', _c_i32),
        ('gevd', _c_i32), ('rank', _c_i32), ('ref', _c_i32), ('families', _c_i32),
        ('alphaExt', ctypes.c_float),
        ('extMode', _p_i32), ('beta', ctypes.POINTER(ctypes.c_double)), ('betaExt', _p_f32),
        ('winAnalysis', _p_f32), ('winSynthesis', _p_f32),
        ('bcEnd', _p_i32), ('upEnd', _p_i32), ('flags', _p_u8),
        ('w0', _p_f32), ('wExt0', _p_f32), ('wExtTarget0', _p_f32), ('scmInit', ctypes.POINTER(ctypes.c_double)),
        ('keepHistory', _c_i32),
        ('zLag', _p_u8), ('zPhase', ctypes.POINTER(ctypes.c_double)),
        ('fsTab', _p_i32), ('zStreamLen', _c_i32), ('scmInitPerBin', _c_i32),
        ('cohDrift', _c_i32), ('cdSegLength', _c_i32), ('cdStart', _c_i32), ('cdEvery', _c_i32),
        ('cdCompensate', _c_i32), ('cdNIter', _c_i32), ('cdAlpha', ctypes.c_double), ('cdAlphaEps', ctypes.c_double),
        ('cEnd', _p_i32), ('cPhase', ctypes.POINTER(ctypes.c_double)), ('dxcp', _c_i32), ('smallDGrid', _c_i32),
        ('fsEv', _p_i32), ('nFsEv', _c_i32), ('fsSteps', _p_i32), ('nFsSteps', _c_i32), ('rawStreams', _c_i32),
        ('desSigConv', _c_i32), ('cdFlagWin', ctypes.POINTER(ctypes.c_double)),
    ]


class DanseBatchCfg(ctypes.Structure):
    _fields_ = [
        ('S', _c_i32), ('K', _c_i32), ('M', _p_i32),
        ('N', _c_i32), ('Ns', _c_i32), ('T', _c_i32),
        ('iters', _c_i32), ('nseg', _c_i32),
        ('gevd', _c_i32), ('rank', _c_i32), ('ref', _c_i32),
        ('alphaExt', ctypes.c_float),
        ('extMode', _p_i32), ('betaExt', _p_f32), ('win', _p_f32),
        ('vad', _p_u8), ('doSolve', _p_u8),
        ('w0', _p_f32), ('wExt0', _p_f32),
        ('costTrim', _c_i32),
        ('k0', _c_i32),
        ('k1', _c_i32),
        ('tgt0', ctypes.c_void_p),
        ('obs', _c_i32),
    ]


BOUT_W, BOUT_WEXT, BOUT_D, BOUT_DHAT, BOUT_COST = 0, 1, 2, 3, 4

# every symbol include/danse_mi355x.h declares, with its ctypes signature
SIGNATURES = {
    'danse_engine_create': (_c_i32, [ctypes.POINTER(DanseCfg), _c_i32, ctypes.POINTER(ctypes.c_void_p)]),
    'danse_engine_destroy': (None, [ctypes.c_void_p]),
    'danse_last_error': (ctypes.c_char_p, [ctypes.c_void_p]),
    'danse_mi355x_build_id': (ctypes.c_char_p, []),
    'danse_engine_set_inputs': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_engine_reset': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_engine_run': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, ctypes.c_void_p, _c_i32]),
    'danse_engine_run_resident': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_engine_set_cond': (_c_i32, [ctypes.c_void_p, _c_i32]),
    'danse_engine_cond': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    'danse_engine_resident_error': (_c_i32, [ctypes.c_void_p, ctypes.POINTER(_c_i32), ctypes.c_void_p]),
    'danse_engine_resident_set_error': (_c_i32, [ctypes.c_void_p, _c_i32]),
    'danse_engine_dxcp_record': (_c_i32, [ctypes.c_void_p, _c_i32]),
    'danse_mi355x_fill': (_c_i32, [ctypes.c_void_p, _c_i32, ctypes.c_size_t, ctypes.c_void_p]),
    'danse_engine_run_steps': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, ctypes.c_void_p]),
    'danse_engine_set_zchunk': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_engine_unpack_zchunk': (_c_i32, [ctypes.c_void_p, _c_i32, ctypes.c_void_p]),
    'danse_engine_dxcp_recorded': (_c_i32, [ctypes.c_void_p, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32),
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]),
    'danse_engine_resident_trace': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]),
    'danse_engine_lanczos_stats': (_c_i32, [ctypes.c_void_p, _p_i32, ctypes.c_size_t]),
    'danse_engine_bcast': (_c_i32, [ctypes.c_void_p, _c_i32, ctypes.c_void_p]),
    'danse_engine_update': (_c_i32, [ctypes.c_void_p, _c_i32, ctypes.c_void_p]),
    'danse_engine_finish': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_engine_set_zspec': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_engine_zspec': (_c_i32, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]),
    'danse_engine_gate': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, _p_i32, _p_i32, _p_i32,
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), _p_i32,
                                   ctypes.c_void_p]),
    'danse_engine_set_flags': (_c_i32, [ctypes.c_void_p, _p_u8, ctypes.c_void_p]),
    'danse_engine_set_gate': (_c_i32, [ctypes.c_void_p, _c_i32, _p_i32, _p_i32, _p_i32, _p_i32,
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    'danse_engine_gate_verdicts': (_c_i32, [ctypes.c_void_p, _p_i32, ctypes.c_void_p]),
    'danse_engine_gate_launch': (_c_i32, [ctypes.c_void_p, _c_i32, ctypes.c_void_p]),
    'danse_engine_sro_estimates': (_c_i32, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double)]),
    'danse_engine_get': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, _c_i32, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_void_p]),
    'danse_engine_put': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, _c_i32, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_void_p]),
    'danse_engine_output_bytes': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, _c_i32, ctypes.POINTER(ctypes.c_size_t)]),
    'danse_wola_analysis': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, ctypes.c_void_p, ctypes.c_void_p, _c_i32, _c_i32,
                                     ctypes.c_void_p, ctypes.c_void_p]),
    'danse_filter_update': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'danse_batch_covmats': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, _c_i32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]),
    'danse_stft': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, ctypes.c_void_p,
                            ctypes.c_void_p, ctypes.c_void_p]),
    'danse_batch_create': (_c_i32, [ctypes.POINTER(DanseBatchCfg), _c_i32, ctypes.POINTER(ctypes.c_void_p)]),
    'danse_batch_destroy': (None, [ctypes.c_void_p]),
    'danse_batch_last_error': (ctypes.c_char_p, [ctypes.c_void_p]),
    'danse_batch_set_inputs': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'danse_batch_run': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_batch_run_iters': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, ctypes.c_void_p]),
    'danse_batch_pack_wext': (_c_i32, [ctypes.c_void_p, _c_i32, ctypes.c_void_p, ctypes.c_void_p]),
    'danse_batch_unpack_wext': (_c_i32, [ctypes.c_void_p, _c_i32, ctypes.c_void_p, ctypes.c_void_p]),
    'danse_batch_output_bytes': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, ctypes.POINTER(ctypes.c_size_t)]),
    'danse_batch_get': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    'danse_batch_set_timing': (_c_i32, [ctypes.c_void_p, _c_i32]),
    'danse_batch_timing': (_c_i32, [ctypes.c_void_p, _c_i32, _c_i32, ctypes.POINTER(ctypes.c_float)]),
    'danse_dxcp_create': (_c_i32, [_c_i32, _c_i32, ctypes.POINTER(ctypes.c_void_p)]),
    'danse_dxcp_destroy': (None, [ctypes.c_void_p]),
    'danse_dxcp_last_error': (ctypes.c_char_p, [ctypes.c_void_p]),
    'danse_dxcp_process': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'danse_dxcp_reset': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p]),
    'danse_dxcp_process_tdoa': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    'danse_cl_dxcp_create': (_c_i32, [_c_i32, _c_i32, _c_i32, ctypes.POINTER(ctypes.c_void_p)]),
    'danse_cl_dxcp_process': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    'danse_tz_create': (_c_i32, [_c_i32, ctypes.c_void_p, ctypes.c_void_p, _c_i32, _c_i32,
                                 ctypes.POINTER(ctypes.c_void_p)]),
    'danse_tz_destroy': (None, [ctypes.c_void_p]),
    'danse_metrics_last_error': (ctypes.c_char_p, []),
    'danse_snr': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, _c_i32,
                           ctypes.c_void_p, ctypes.c_void_p]),
    'danse_fwsnrseg_frames': (_c_i32, [ctypes.c_int64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.POINTER(_c_i32)]),
    'danse_fwsnrseg': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, _c_i32, ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p]),
    'danse_scene_last_error': (ctypes.c_char_p, []),
    'danse_scene_generate': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    'danse_scene_convolve_vad': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, _c_i32, _c_i32, _c_i32, ctypes.c_void_p,
                                          ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    'danse_stoi_last_error': (ctypes.c_char_p, []),
    'danse_stoi': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, _c_i32, ctypes.c_double, _c_i32,
                            ctypes.c_void_p, ctypes.c_void_p]),
    'danse_tz_last_error': (ctypes.c_char_p, [ctypes.c_void_p]),
    'danse_tz_ir': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, _c_i32, _c_i32, ctypes.c_void_p, ctypes.c_void_p]),
    'danse_tz_compress': (_c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _c_i32, _c_i32, _c_i32,
                                   ctypes.c_void_p, ctypes.c_void_p]),
}

_lib = None


def load_library(path: os.PathLike | None = None):
    """Load (once) and type the HIP library.  Raises if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise RuntimeError(f'{p} not found: build the HIP extension first (python -c "import __graft_entry__ as g; g.build()")')
    lib = ctypes.CDLL(str(p))
    _check_build_id(lib, p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _check_build_id(lib, p: Path) -> None:
    """The library must be the build of the sources next to it (build.py
    embeds their hash).  Without sources (an installed copy) there is nothing
    to compare.  DANSE_LIB points at A/B variants, which carry their own."""
    from . import build as _b
    if not _b.CSRC.exists():
        return
    fn = lib.danse_mi355x_build_id
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    have = (fn() or b'').decode()
    name = p.name
    variant = name[len('libdanse_'):-3] if name.startswith('libdanse_') and name != LIB_NAME else None
    want = _b.source_hash(variant if variant in _b.VARIANTS else None)
    if have != want:
        raise RuntimeError(f'{p} was built from other sources (build id {have[:16]}, sources {want[:16]}): '
                           'rebuild it (python -c "import __graft_entry__ as g; g.build()")')


class DanseError(RuntimeError):
    pass


def check(rc: int, eng=None):
    if rc != 0:
        lib = load_library()
        msg = lib.danse_last_error(eng)
        raise DanseError((msg or b'').decode() or f'error {rc}')


def check_batch(rc: int, eng=None):
    if rc != 0:
        lib = load_library()
        msg = lib.danse_batch_last_error(eng)
        raise DanseError((msg or b'').decode() or f'error {rc}')
