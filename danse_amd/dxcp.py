"""DXCP-PhaT sampling-rate-offset estimation on the device (SURVEY §8a row
a12; ``dxcpphat/sro_estimation.py:130-345``), batched over node pairs.

``DXCPPhaT`` mirrors the reference class with its default parameters
(``process_data(x_12_ell)`` with ``x_12_ell`` of shape (2048, 2), returning
``{'SROppm_est_out', 'STOsmp_est_out'}``); ``DXCPPhaTBatch`` runs P pairs per
call (``process_frames`` with frames of shape (P, 2, 2048)).  The estimator
state (input ring, GCSD-PhaT average, 40-frame container, CSD-2 and CCF-1
averages) stays in HBM between calls.  No CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L

FRAME = 2048


class DXCPPhaTBatch:
    def __init__(self, P: int, device: int = 0):
        import torch
        self.torch = torch
        self.lib = L.load_library()
        self.P = int(P)
        self.device = device
        eng = ctypes.c_void_p()
        rc = self.lib.danse_dxcp_create(self.P, int(device), ctypes.byref(eng))
        if rc != 0:
            raise L.DanseError((self.lib.danse_dxcp_last_error(None) or b'').decode() or f'error {rc}')
        self.eng = eng
        self._x = torch.zeros((self.P, 2, FRAME), dtype=torch.float32, device=f'cuda:{device}')
        self._out = torch.zeros((self.P, 2), dtype=torch.float64, device=f'cuda:{device}')

    def process_frames(self, frames, stream=None):
        """frames: (P, 2, 2048) array or device tensor.  Returns (sro_ppm,
        sto_samples) device tensors of shape (P,) after this frame."""
        t = self.torch
        if isinstance(frames, t.Tensor) and frames.is_cuda and frames.dtype == t.float32 and frames.is_contiguous():
            x = frames
        else:
            self._x.copy_(t.as_tensor(np.asarray(frames, dtype=np.float32)).reshape(self.P, 2, FRAME))
            x = self._x
        st = stream if stream is not None else t.cuda.current_stream(self.device)
        rc = self.lib.danse_dxcp_process(self.eng, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(self._out.data_ptr()),
                                         ctypes.c_void_p(st.cuda_stream))
        if rc != 0:
            raise L.DanseError((self.lib.danse_dxcp_last_error(self.eng) or b'').decode() or f'error {rc}')
        return self._out[:, 0], self._out[:, 1]

    def close(self):
        if getattr(self, 'eng', None):
            self.lib.danse_dxcp_destroy(self.eng)
            self.eng = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DXCPPhaT:
    """Single-pair drop-in of the reference's ``DXCPPhaT`` (default params)."""

    def __init__(self, device: int = 0):
        self._b = DXCPPhaTBatch(1, device=device)

    def process_data(self, x_12_ell, tdoa=0):
        if tdoa != 0:
            raise NotImplementedError('tdoa correction of the STO estimate')
        x = np.asarray(x_12_ell, dtype=np.float32).T.reshape(1, 2, FRAME)
        sro, sto = self._b.process_frames(x)
        return {'SROppm_est_out': float(sro[0].item()), 'STOsmp_est_out': float(sto[0].item())}
