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

    def _frames(self, frames):
        t = self.torch
        if isinstance(frames, t.Tensor) and frames.is_cuda and frames.dtype == t.float32 and frames.is_contiguous():
            return frames
        self._x.copy_(t.as_tensor(np.asarray(frames, dtype=np.float32)).reshape(self.P, 2, FRAME))
        return self._x

    def process_frames(self, frames, tdoa=None, stream=None):
        """frames: (P, 2, 2048) array or device tensor; tdoa: None or (P,)
        seconds (STO correction, sro_estimation.py:338-339).  Returns
        (sro_ppm, sto_samples) device tensors of shape (P,) after this frame."""
        t = self.torch
        x = self._frames(frames)
        st = stream if stream is not None else t.cuda.current_stream(self.device)
        if tdoa is None:
            rc = self.lib.danse_dxcp_process(self.eng, ctypes.c_void_p(x.data_ptr()),
                                             ctypes.c_void_p(self._out.data_ptr()), ctypes.c_void_p(st.cuda_stream))
        else:
            td = t.as_tensor(np.broadcast_to(np.asarray(tdoa, dtype=np.float64), (self.P,)).copy()).to(x.device)
            rc = self.lib.danse_dxcp_process_tdoa(self.eng, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(td.data_ptr()),
                                                  ctypes.c_void_p(self._out.data_ptr()), ctypes.c_void_p(st.cuda_stream))
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
        x = np.asarray(x_12_ell, dtype=np.float32).T.reshape(1, 2, FRAME)
        sro, sto = self._b.process_frames(x, tdoa=None if tdoa == 0 else [tdoa])
        return {'SROppm_est_out': float(sro[0].item()), 'STOsmp_est_out': float(sto[0].item())}


class CL_DXCPPhaTBatch:
    """P closed-loop DXCP-PhaT estimators (``CL_DXCPPhaT``,
    ``sro_estimation.py:12-72``) on the device: resampler, delay buffer,
    DXCP-PhaT and IMC controller state stay in HBM."""

    def __init__(self, P: int, start_delay: int = 0, device: int = 0):
        import torch
        self.torch = torch
        self.lib = L.load_library()
        self.P = int(P)
        self.device = device
        eng = ctypes.c_void_p()
        rc = self.lib.danse_cl_dxcp_create(self.P, int(start_delay), int(device), ctypes.byref(eng))
        if rc != 0:
            raise L.DanseError((self.lib.danse_dxcp_last_error(None) or b'').decode() or f'error {rc}')
        self.eng = eng
        dev = f'cuda:{device}'
        self._x = torch.zeros((self.P, 2, FRAME), dtype=torch.float32, device=dev)
        self._acs = torch.ones((self.P,), dtype=torch.int32, device=dev)
        self.out = torch.zeros((self.P, 3), dtype=torch.float64, device=dev)
        self.zi = torch.zeros((self.P, FRAME), dtype=torch.float32, device=dev)

    def process_frames(self, frames, acs=None, stream=None):
        """frames: (P, 2, 2048) (z_j, z_i); acs: None or (P,) 0/1.  Returns
        the (P, 3) device tensor (raw residual ppm, SRO estimate ppm, shift)
        and the (P, 2048) synchronised z_i blocks."""
        t = self.torch
        if isinstance(frames, t.Tensor) and frames.is_cuda and frames.dtype == t.float32 and frames.is_contiguous():
            x = frames
        else:
            self._x.copy_(t.as_tensor(np.asarray(frames, dtype=np.float32)).reshape(self.P, 2, FRAME))
            x = self._x
        a = None
        if acs is not None:
            self._acs.copy_(t.as_tensor(np.broadcast_to(np.asarray(acs, dtype=np.int32), (self.P,)).copy()))
            a = self._acs
        st = stream if stream is not None else t.cuda.current_stream(self.device)
        rc = self.lib.danse_cl_dxcp_process(self.eng, ctypes.c_void_p(x.data_ptr()),
                                            ctypes.c_void_p(a.data_ptr()) if a is not None else None,
                                            ctypes.c_void_p(self.out.data_ptr()), ctypes.c_void_p(self.zi.data_ptr()),
                                            ctypes.c_void_p(st.cuda_stream))
        if rc != 0:
            raise L.DanseError((self.lib.danse_dxcp_last_error(self.eng) or b'').decode() or f'error {rc}')
        return self.out, self.zi

    def close(self):
        if getattr(self, 'eng', None):
            self.lib.danse_dxcp_destroy(self.eng)
            self.eng = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CL_DXCPPhaT:
    """Single-pair drop-in of the reference's ``CL_DXCPPhaT``:
    ``process(x_12_ell, acs)`` returns (dSRO_est_curr_raw, SRO_est_curr,
    Resampler.shift, z_i)."""

    def __init__(self, start_delay=0, device: int = 0):
        self._b = CL_DXCPPhaTBatch(1, start_delay=start_delay, device=device)

    def process(self, x_12_ell, acs=1):
        x = np.asarray(x_12_ell, dtype=np.float32).T.reshape(1, 2, FRAME)
        out, zi = self._b.process_frames(x, acs=[acs])
        o = out.cpu().numpy()[0]
        return float(o[0]), float(o[1]), float(o[2]), zi.cpu().numpy()[0].astype(np.float64)
