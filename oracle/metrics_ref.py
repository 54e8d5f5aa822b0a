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


# --------------------------------------------------------------------------- #
# (e)STOI -- danse_toolbox/mypystoi/stoi.py:18-239, utils.py (pystoi).
# Restated without the EPS-level random perturbation of row_col_normalize
# (utils.py:134-149: EPS * np.random.standard_normal, ~1e-16 relative).
# --------------------------------------------------------------------------- #
STOI_FS = 10000
STOI_NFRAME = 256
STOI_NFFT = 512
STOI_NUMBAND = 15
STOI_MINFREQ = 150
STOI_N = 30
STOI_BETA = -15.0
STOI_DYN = 40
EPS = np.finfo('float').eps


def thirdoct(fs=STOI_FS, nfft=STOI_NFFT, num_bands=STOI_NUMBAND, min_freq=STOI_MINFREQ):
    """utils.py:57-84: the bin range [lo, hi) of every 1/3-octave band."""
    f = np.linspace(0, fs, nfft + 1)[:nfft // 2 + 1]
    k = np.arange(num_bands).astype(float)
    lo = min_freq * np.power(2., (2 * k - 1) / 6)
    hi = min_freq * np.power(2., (2 * k + 1) / 6)
    out = np.zeros((num_bands, 2), dtype=np.int64)
    for i in range(num_bands):
        out[i, 0] = np.argmin(np.square(f - lo[i]))
        out[i, 1] = np.argmin(np.square(f - hi[i]))
    return out


def resample_window_oct(p, q):
    """utils.py:8-40 (Kaiser-windowed sinc of the Octave resampler)."""
    g = np.gcd(p, q)
    p, q = p // g, q // g
    log10_rejection = -3.0
    stop = 1. / (2 * max(p, q))
    roll = stop / 10
    rej = -20 * log10_rejection
    L = np.ceil((rej - 8) / (28.714 * roll))
    t = np.arange(-L, L + 1)
    ideal = 2 * p * stop * np.sinc(2 * stop * t)
    if 21 <= rej <= 50:
        beta = 0.5842 * (rej - 21) ** 0.4 + 0.07886 * (rej - 21)
    elif rej > 50:
        beta = 0.1102 * (rej - 8.7)
    else:
        beta = 0.0
    return np.kaiser(2 * L + 1, beta) * ideal


def resample_oct(x, p, q):
    """utils.py:43-47: resample_poly(x, p, q) with that window (sum-normalised)."""
    from scipy.signal import resample_poly
    h = resample_window_oct(p, q)
    return resample_poly(x, p, q, window=h / np.sum(h))


def _hann(n):
    return np.hanning(n + 2)[1:-1]


def remove_silent_frames(x, y, dyn_range=STOI_DYN, framelen=STOI_NFRAME, hop=STOI_NFRAME // 2):
    """utils.py:102-126."""
    w = _hann(framelen)
    xf = np.array([w * x[i:i + framelen] for i in range(0, len(x) - framelen, hop)])
    yf = np.array([w * y[i:i + framelen] for i in range(0, len(x) - framelen, hop)])
    e = 20 * np.log10(np.linalg.norm(xf, axis=1) + EPS)
    mask = (np.max(e) - dyn_range - e) < 0
    xf, yf = xf[mask], yf[mask]
    n = (len(xf) - 1) * hop + framelen
    xs, ys = np.zeros(n), np.zeros(n)
    for i in range(xf.shape[0]):
        xs[i * hop:i * hop + framelen] += xf[i]
        ys[i * hop:i * hop + framelen] += yf[i]
    return xs, ys


def stoi_stft(x, win=STOI_NFRAME, nfft=STOI_NFFT, overlap=2):
    """utils.py:87-99."""
    hop = int(win / overlap)
    w = _hann(win)
    return np.array([np.fft.rfft(w * x[i:i + win], n=nfft) for i in range(0, len(x) - win, hop)])


def stoi(x, y, fs_sig, extended=False):
    """stoi.py:18-119 (``stoi``; resample_oct to 10 kHz) -- and, at
    fs_sig == 10000, ``stoi_any_fs`` (stoi.py:122-239), whose only
    difference is resampy for fs_sig != 10000."""
    x = np.squeeze(np.asarray(x, dtype=np.float64))
    y = np.squeeze(np.asarray(y, dtype=np.float64))
    if fs_sig != STOI_FS:
        x = resample_oct(x, STOI_FS, int(fs_sig))
        y = resample_oct(y, STOI_FS, int(fs_sig))
    x, y = remove_silent_frames(x, y)
    xs = stoi_stft(x).T
    ys = stoi_stft(y).T
    if xs.shape[-1] < STOI_N:
        return 1e-5
    bands = thirdoct()
    obm = np.zeros((STOI_NUMBAND, STOI_NFFT // 2 + 1))
    for i, (lo, hi) in enumerate(bands):
        obm[i, lo:hi] = 1
    xt = np.sqrt(obm @ np.square(np.abs(xs)))
    yt = np.sqrt(obm @ np.square(np.abs(ys)))
    xseg = np.array([xt[:, m - STOI_N:m] for m in range(STOI_N, xt.shape[1] + 1)])
    yseg = np.array([yt[:, m - STOI_N:m] for m in range(STOI_N, xt.shape[1] + 1)])
    if extended:
        def rcn(a):
            a = a - np.mean(a, axis=-1, keepdims=True)
            a = a / np.sqrt(np.sum(np.square(a), axis=-1, keepdims=True))
            a = a - np.mean(a, axis=1, keepdims=True)
            return a / np.sqrt(np.sum(np.square(a), axis=1, keepdims=True))
        xn, yn = rcn(xseg), rcn(yseg)
        return np.sum(xn * yn / STOI_N) / xn.shape[0]
    nc = np.linalg.norm(xseg, axis=2, keepdims=True) / (np.linalg.norm(yseg, axis=2, keepdims=True) + EPS)
    yp = np.minimum(yseg * nc, xseg * (1 + 10 ** (-STOI_BETA / 20)))
    yp = yp - np.mean(yp, axis=2, keepdims=True)
    xs_ = xseg - np.mean(xseg, axis=2, keepdims=True)
    yp /= (np.linalg.norm(yp, axis=2, keepdims=True) + EPS)
    xs_ /= (np.linalg.norm(xs_, axis=2, keepdims=True) + EPS)
    return np.sum(yp * xs_) / (xs_.shape[0] * xs_.shape[1])
