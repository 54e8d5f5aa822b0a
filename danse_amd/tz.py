"""T(z) few-samples compression on the device (SURVEY §8a row a14;
``danse_tz_*`` C-ABI, ``csrc/tz.hip``).

``TZCompressor`` runs B nodes per launch: ``ir`` is ``dist_fct_approx``
(``danse_toolbox/d_base.py:1941-1991``) and ``compress`` the convolution of
``danse_compression_few_samples`` (``d_base.py:1871-1938``).  The module-level
``dist_fct_approx`` / ``danse_compression_few_samples`` keep the reference's
signatures and array layouts for one node (host arrays in, host arrays out).
No CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


class TZCompressor:
    def __init__(self, h, f, R: int, device: int = 0):
        import torch
        self.torch = torch
        self.lib = L.load_library()
        h = np.ascontiguousarray(h, dtype=np.float32)
        f = np.ascontiguousarray(f, dtype=np.float32)
        if h.shape != f.shape or h.ndim != 1:
            raise ValueError('h and f must be 1-D windows of the same length')
        self.N = len(h)
        self.device = device
        eng = ctypes.c_void_p()
        rc = self.lib.danse_tz_create(self.N, h.ctypes.data_as(ctypes.c_void_p), f.ctypes.data_as(ctypes.c_void_p),
                                      int(R), int(device), ctypes.byref(eng))
        if rc != 0:
            raise L.DanseError((self.lib.danse_tz_last_error(None) or b'').decode() or f'error {rc}')
        self.eng = eng

    def _check(self, rc):
        if rc != 0:
            raise L.DanseError((self.lib.danse_tz_last_error(self.eng) or b'').decode() or f'error {rc}')

    def _stream(self, stream):
        st = stream if stream is not None else self.torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(st.cuda_stream)

    def _dev(self, x, dtype):
        t = self.torch
        if isinstance(x, t.Tensor):
            x = x.to(device=f'cuda:{self.device}', dtype=dtype)
        else:
            x = t.as_tensor(np.asarray(x), dtype=dtype, device=f'cuda:{self.device}')
        return x.contiguous()

    def ir(self, wHat, out=None, stream=None):
        """wHat: (B, N/2+1, M) complex -> wIR (B, 2N-1, M) float32 device tensor."""
        t = self.torch
        w = self._dev(wHat, t.complex64)
        if w.ndim != 3 or w.shape[1] != self.N // 2 + 1:
            raise ValueError(f'wHat must be (B, {self.N // 2 + 1}, M)')
        B, _, M = w.shape
        if out is None:
            out = t.empty((B, 2 * self.N - 1, M), dtype=t.float32, device=w.device)
        self._check(self.lib.danse_tz_ir(self.eng, ctypes.c_void_p(w.data_ptr()), B, M,
                                         ctypes.c_void_p(out.data_ptr()), self._stream(stream)))
        return out

    def compress(self, yq, wIR, L_: int, out=None, stream=None):
        """yq: (B, N, M) frames, wIR: (B, 2N-1, M) -> z (B, L) float32 device tensor."""
        t = self.torch
        y = self._dev(yq, t.float32)
        a = self._dev(wIR, t.float32)
        if y.ndim != 3 or y.shape[1] != self.N or a.shape != (y.shape[0], 2 * self.N - 1, y.shape[2]):
            raise ValueError('yq must be (B, N, M) and wIR (B, 2N-1, M)')
        B, _, M = y.shape
        if out is None:
            out = t.empty((B, int(L_)), dtype=t.float32, device=y.device)
        self._check(self.lib.danse_tz_compress(self.eng, ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(a.data_ptr()),
                                               B, M, int(L_), ctypes.c_void_p(out.data_ptr()), self._stream(stream)))
        return out

    def close(self):
        if getattr(self, 'eng', None):
            self.lib.danse_tz_destroy(self.eng)
            self.eng = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dist_fct_approx(wHat, h, f, R, device=0):
    """``d_base.py:1941-1991`` for one node: wHat (N/2+1, M) -> (2N-1, M)."""
    c = TZCompressor(h, f, R, device)
    w = np.asarray(wHat)
    return c.ir(w.reshape(1, *w.shape)).cpu().numpy()[0].astype(np.float64)


def danse_compression_few_samples(yq, wqqHat, L_, wIRprevious, winWOLAanalysis, winWOLAsynthesis, Ns,
                                  updateBroadcastFilter=False, device=0):
    """``d_base.py:1871-1938`` for one node: returns (zq (L,), wIR (2N-1, M))."""
    c = TZCompressor(winWOLAanalysis, winWOLAsynthesis, Ns, device)
    yq = np.asarray(yq)
    if updateBroadcastFilter:
        w = np.asarray(wqqHat)
        wIR = c.ir(w.reshape(1, *w.shape))
    else:
        wIR = c._dev(np.asarray(wIRprevious)[None], c.torch.float32)
    z = c.compress(yq.reshape(1, *yq.shape), wIR, L_)
    return z.cpu().numpy()[0].astype(np.float64), wIR.cpu().numpy()[0].astype(np.float64)
