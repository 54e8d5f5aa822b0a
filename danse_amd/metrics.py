"""Enhancement metrics on the device (``danse_snr`` /
``danse_fwsnrseg`` C-ABI, ``csrc/metrics.hip``), float64 like the reference.

* ``get_snr(s, n, vad=None, bypassVADuse=False)`` -- ``get_snr``
  (``danse_toolbox/d_eval.py:573-624``), same argument layout ([T x C] or
  1-D host arrays) and return type (float for one channel).
* ``get_fwsnrseg(cleanSig, enhancedSig, fs, frameLen=0.03, overlap=0.75,
  gamma=0.2)`` -- ``get_fwsnrseg`` (``d_eval.py:660-778``): the per-frame
  values of one signal pair.
* ``fwsnrseg_batch(clean, enhanced, fs, ...)`` -- device tensors [B][T] in,
  per-frame [B][nFrames] and mean [B] device tensors out (the E battery's
  ΔfwSNRseg per scene without leaving the GPU).
No CPU fallback: the library must be present.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


def _check(rc):
    if rc != 0:
        lib = L.load_library()
        raise L.DanseError((lib.danse_metrics_last_error() or b'').decode() or f'error {rc}')


def _dev(x, torch, device):
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))
    return t.to(device=device, dtype=torch.float64).contiguous()


def _stream(torch, device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def fwsnrseg_frames(T, fs, frameLen=0.03, overlap=0.75):
    lib = L.load_library()
    nf = ctypes.c_int32()
    _check(lib.danse_fwsnrseg_frames(int(T), float(fs), float(frameLen), float(overlap), ctypes.byref(nf)))
    return nf.value


def fwsnrseg_batch(clean, enhanced, fs, frameLen=0.03, overlap=0.75, gamma=0.2, device=0):
    """clean, enhanced: [B][T] (device tensors or host arrays).  Returns
    (perFrame [B][nFrames], mean [B]) float64 device tensors."""
    import torch
    lib = L.load_library()
    dev = f'cuda:{device}'
    c = _dev(clean, torch, dev)
    e = _dev(enhanced, torch, dev)
    if c.ndim == 1:
        c, e = c[None], e[None]
    if c.shape != e.shape:
        raise ValueError('The two signals do not match!')
    B, T = c.shape
    nf = fwsnrseg_frames(T, fs, frameLen, overlap)
    per = torch.empty((B, nf), dtype=torch.float64, device=dev)
    mean = torch.empty((B,), dtype=torch.float64, device=dev)
    _check(lib.danse_fwsnrseg(ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(e.data_ptr()), T, B, float(fs),
                              float(frameLen), float(overlap), float(gamma), ctypes.c_void_p(per.data_ptr()),
                              ctypes.c_void_p(mean.data_ptr()), _stream(torch, dev)))
    return per, mean


def get_fwsnrseg(cleanSig, enhancedSig, fs, frameLen=0.03, overlap=0.75, gamma=0.2):
    """The reference's signature: 1-D signals (or [T x 1] with 1-D), per-frame values (numpy)."""
    c = np.asarray(cleanSig, dtype=np.float64)
    e = np.asarray(enhancedSig, dtype=np.float64)
    if c.ndim == 2 and e.ndim == 1:
        c = c[:, 0]
    if c.ndim == 1 and e.ndim == 2:
        e = e[:, 0]
    if c.shape != e.shape:
        raise ValueError('The two signals do not match!')
    per, _ = fwsnrseg_batch(c[None], e[None], fs, frameLen, overlap, gamma)
    return per[0].cpu().numpy()


def get_snr(s, n, vad=None, bypassVADuse=False, device=0):
    import torch
    lib = L.load_library()
    s = np.asarray(s, dtype=np.float64)
    n = np.asarray(n, dtype=np.float64)
    if s.ndim == 1:
        s = s[:, None]
    if n.ndim == 1:
        n = n[:, None]
    if s.shape != n.shape:
        raise ValueError('s and n must have the same shape')
    T, C = s.shape
    dev = f'cuda:{device}'
    sd = _dev(s.T, torch, dev)
    nd = _dev(n.T, torch, dev)
    vd = None
    if vad is not None and not bypassVADuse:
        v = np.asarray(vad)
        if v.ndim == 1:
            v = v[:, None]
        v = np.broadcast_to(v.astype(bool), (T, C))
        vd = torch.from_numpy(np.ascontiguousarray(v.T.astype(np.uint8))).to(dev)
    out = torch.empty((C,), dtype=torch.float64, device=dev)
    _check(lib.danse_snr(ctypes.c_void_p(sd.data_ptr()), ctypes.c_void_p(nd.data_ptr()),
                         ctypes.c_void_p(vd.data_ptr()) if vd is not None else None, T, C,
                         ctypes.c_void_p(out.data_ptr()), _stream(torch, dev)))
    o = out.cpu().numpy()
    return float(o[0]) if C == 1 else o
