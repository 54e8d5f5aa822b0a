"""TEST INFRASTRUCTURE ONLY (the checker, never the product): float64 NumPy
restatement of the reference's enhancement metrics, used by tests/ to check
the device kernels of danse_amd/csrc/metrics.hip.

* ``get_snr``       -- danse_toolbox/d_eval.py:573-624
* ``get_fwsnrseg``  -- danse_toolbox/d_eval.py:660-778 (adapted from pysepm:
  25 critical bands, Hann frames of round(frameLen fs) samples every
  floor((1 - overlap) frameLen fs), nfft = 2^ceil(log2(2 W)), magnitude
  spectra normalised per frame over bins 0..nfft/2-1, weighted log-SNR,
  clipped to [0, 35] dB).  The reference calls scipy.signal.stft; its
  1/sum(window) scaling cancels in the per-frame normalisation, so the
  frames here go through np.fft.rfft directly.

Pinned by tests/golden/metrics_*.npz (the reference's own functions run on
the same inputs, tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np

CENT = np.array([50.0000, 120.000, 190.000, 260.000, 330.000, 400.000, 470.000, 540.000, 617.372, 703.378, 798.717,
                 904.128, 1020.38, 1148.30, 1288.72, 1442.54, 1610.70, 1794.16, 1993.93, 2211.08, 2446.71, 2701.97,
                 2978.04, 3276.17, 3597.63])
BW = np.array([70.0000, 70.0000, 70.0000, 70.0000, 70.0000, 70.0000, 70.0000, 77.3724, 86.0056, 95.3398, 105.411,
               116.256, 127.914, 140.423, 153.823, 168.154, 183.457, 199.776, 217.153, 235.631, 255.255, 276.072,
               298.126, 321.465, 346.136])


def get_snr(s, n, vad=None, bypassVADuse=False):
    """d_eval.py:573-624: 10 log10(mean |s|^2 / mean |n|^2) over the VAD, per channel."""
    s = np.asarray(s)
    n = np.asarray(n)
    if vad is None or bypassVADuse:
        vad = np.ones(s.shape, dtype=bool)
    if s.ndim == 1:
        s = s[:, None]
    if n.ndim == 1:
        n = n[:, None]
    vad = np.asarray(vad)
    if vad.ndim == 1:
        vad = vad[:, None]
    vad = vad.astype(bool)
    out = np.array([10 * np.log10(np.mean(np.abs(s[vad[:, c], c]) ** 2) / np.mean(np.abs(n[vad[:, c], c]) ** 2))
                    for c in range(s.shape[-1])])
    return out[0] if s.shape[-1] == 1 else out


def fw_frames(T, fs, frameLen=0.03, overlap=0.75):
    """(W, skip, nfft, nFrames) as d_eval.py:676-679,737."""
    W = round(frameLen * fs)
    skip = int(np.floor((1 - overlap) * frameLen * fs))
    nfft = int(2 ** np.ceil(np.log2(2 * W)))
    nf = int(T / skip - (W / skip))
    return W, skip, nfft, nf


def crit_filters(fs, nfft):
    """d_eval.py:719-733."""
    h = nfft // 2
    maxf = fs / 2
    minf = np.exp(-30.0 / (2.0 * 2.303))
    j = np.arange(0, h)
    cf = np.zeros((len(CENT), h))
    for i in range(len(CENT)):
        f0 = (CENT[i] / maxf) * h
        bw = (BW[i] / maxf) * h
        nrm = np.log(BW[0]) - np.log(BW[i])
        cf[i] = np.exp(-11 * (((j - np.floor(f0)) / bw) ** 2) + nrm)
        cf[i] = cf[i] * (cf[i] > minf)
    return cf


def get_fwsnrseg(cleanSig, enhancedSig, fs, frameLen=0.03, overlap=0.75, gamma=0.2):
    """d_eval.py:660-778: per-frame frequency-weighted segmental SNR [dB]."""
    eps = np.finfo(np.float64).eps
    c = np.asarray(cleanSig, dtype=np.float64).ravel() + eps
    e = np.asarray(enhancedSig, dtype=np.float64).ravel() + eps
    if c.shape != e.shape:
        raise ValueError('The two signals do not match!')
    W, skip, nfft, nf = fw_frames(len(c), fs, frameLen, overlap)
    win = 0.5 * (1 - np.cos(2 * np.pi * np.arange(1, W + 1) / (W + 1)))
    idx = np.arange(nf)[:, None] * skip + np.arange(W)[None, :]
    cs = np.abs(np.fft.rfft(c[idx] * win, nfft, axis=1))[:, :-1].T     # [nfft/2][nf]
    es = np.abs(np.fft.rfft(e[idx] * win, nfft, axis=1))[:, :-1].T
    cs = cs / cs.sum(0)
    es = es / es.sum(0)
    cf = crit_filters(fs, nfft)
    ce = cf.dot(cs)
    pe = cf.dot(es)
    err = np.power(ce - pe, 2)
    err[err < eps] = eps
    wf = np.power(ce, gamma)
    snrlog = 10 * np.log10((ce ** 2) / err)
    fw = np.sum(wf * snrlog, 0) / np.sum(wf, 0)
    return np.clip(fw, 0, 35)
