"""TEST INFRASTRUCTURE ONLY -- float64 NumPy restatement of the device scene
generator (danse_amd/csrc/scene.hip), the random-IR / random-signal path of
the reference's siggen (trueRoom false, signalType random):

* counter-based uniform draws (splitmix64 of (seed + scene, stream, index)),
  bit-identical to the device's;
* paused desired source and uniform noise source (siggen/classes.py:32-64);
* uniform [-0.5, 0.5] IRs and causal convolution (siggen/utils.py:229-308);
* noise gain for the SNR at mic 0 of node 0 (siggen/utils.py:1421-1431);
* SRO resampling to fs (1 + SRO 1e-6) with the Kaiser-windowed sinc of the
  device (the reference's resample_for_sro, siggen/utils.py:1579-1622, uses
  resampy, absent offline -- this resampler is parity unpinned against it);
* white self-noise per sensor (siggen/utils.py:1414-1431);
* energy VAD of each node's mic-0 wet speech (oracleVAD, siggen/utils.py:
  1079-1151), pinned with the wet-signal convolution to the reference's own
  get_vad on injected inputs (tests/golden/scene_vad_conv.npz).

The device accumulates the convolution in float32 and rounds every output
to float32; tests compare at a relative tolerance.
"""
from __future__ import annotations

import numpy as np
from scipy.signal import fftconvolve

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
ST_DESIRED, ST_NOISE, ST_IRS, ST_IRN, ST_SELF = 1, 2, 3, 4, 5


def _u64(x):
    return np.asarray(x, dtype=np.uint64)


def mix64(z):
    with np.errstate(over='ignore'):
        z = _u64(z) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream_key(seed, a, b, c):
    with np.errstate(over='ignore'):
        x = mix64(mix64(_u64(seed)) ^ (_u64(a) * np.uint64(0x9E3779B1)))
        return mix64(x ^ (_u64(b) * np.uint64(0x85EBCA77) + _u64(c) * np.uint64(0xC2B2AE3D) + np.uint64(1)))


def urand(key, n):
    """uniform [-1, 1) draws 0 .. n-1 of the stream `key`."""
    with np.errstate(over='ignore'):
        i = np.arange(n, dtype=np.uint64) + np.uint64(0x632BE59BD9B4E019)
        r = mix64(_u64(key) ^ mix64(i))
    return (r >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def resample_sro(x, eps, half=32, roll=0.95, beta=8.0):
    """y[n] = x(n / (1 + eps)) by the Kaiser-windowed sinc of scene.hip."""
    T = len(x)
    if eps == 0.0:
        return x.copy()
    out = np.zeros(T)
    outLen = int(np.ceil(T * (1.0 + eps)))
    fc = min(1.0, 1.0 + eps) * roll
    i0b = np.i0(beta)
    n = np.arange(min(T, outLen))
    p = n / (1.0 + eps)
    base = np.floor(p).astype(np.int64)
    for o in range(-half + 1, half + 1):
        i = base + o
        ok = (i >= 0) & (i < T)
        u = p - i
        r2 = u / half
        ok &= np.abs(r2) < 1.0
        a = np.pi * fc * u
        sinc = np.where(u == 0.0, 1.0, np.sin(a) / np.where(a == 0.0, 1.0, a))
        w = np.i0(beta * np.sqrt(np.clip(1.0 - r2 * r2, 0.0, None))) / i0b
        out[n] += np.where(ok, x[np.clip(i, 0, T - 1)] * fc * sinc * w, 0.0)
    return out


def energy_vad(x, fs, tw, dB):
    """oracleVAD + compute_VAD (siggen/utils.py:1079-1151) with the
    threshold of get_or_load_vad (utils.py:921): sample i is active when the
    MEAN energy of x[max(i - nw//2, 0) : min(i + nw//2, n)] exceeds
    max(x^2) / 10^(dB/10), nw = int(tw fs)."""
    thr = np.max(x ** 2) / 10 ** (dB / 10)
    nw = max(int(tw * fs), 1)
    c = np.concatenate(([0.0], np.cumsum(x ** 2)))
    idx = np.arange(len(x))
    b = np.maximum(idx - nw // 2, 0)
    e = np.minimum(idx + nw // 2, len(x))
    return ((c[e] - c[b]) / (e - b) > thr).astype(np.uint8)


def wet_signal(x, h):
    """sig.fftconvolve(xdry, rir)[:N] (get_vad, siggen/utils.py:867-872)."""
    return fftconvolve(x, h)[:len(x)]


def generate(M, S, T, nIR, seed, fs=16000.0, snr=5.0, selfnoiseSNR=15.0, pauseDuration=0.5, pauseSpacing=0.5,
             vadEnergyDecrease_dB=40.0, vadWinLength=0.04, sroPpm=None):
    """(data, cleanspeech, cleannoise [S][sum M][T], vad [S][K][T])."""
    K = len(M)
    MT = int(sum(M))
    chan = [(k, m) for k in range(K) for m in range(M[k])]
    base = np.concatenate(([0], np.cumsum(M)[:-1])).astype(int)
    sro = np.zeros(K) if sroPpm is None else np.asarray(sroPpm, dtype=np.float64)
    data = np.zeros((S, MT, T))
    cs = np.zeros((S, MT, T))
    cn = np.zeros((S, MT, T))
    vad = np.zeros((S, K, T), dtype=np.uint8)
    t = np.arange(T) / fs
    for s in range(S):
        sd = seed + s
        d = urand(stream_key(sd, ST_DESIRED, 0, 0), T).astype(np.float32).astype(np.float64)
        d[np.fmod(t, pauseDuration + pauseSpacing) >= pauseSpacing] = 0.0
        n = urand(stream_key(sd, ST_NOISE, 0, 0), T).astype(np.float32).astype(np.float64)
        wS = np.zeros((MT, T))
        wN = np.zeros((MT, T))
        for c, (k, m) in enumerate(chan):
            hS = (0.5 * urand(stream_key(sd, ST_IRS, k, m), nIR)).astype(np.float32).astype(np.float64)
            hN = (0.5 * urand(stream_key(sd, ST_IRN, k, m), nIR)).astype(np.float32).astype(np.float64)
            wS[c] = wet_signal(d, hS)
            wN[c] = wet_signal(n, hN)
        gN = 10 ** (-(snr - 10 * np.log10(np.mean(wS[0] ** 2) / np.mean(wN[0] ** 2))) / 20)
        for k in range(K):
            vad[s, k] = energy_vad(wS[base[k]], fs, vadWinLength, vadEnergyDecrease_dB)
        rS = np.stack([resample_sro(wS[c], sro[k] * 1e-6) for c, (k, m) in enumerate(chan)])
        rN = np.stack([resample_sro(wN[c], sro[k] * 1e-6) for c, (k, m) in enumerate(chan)])
        sn = np.zeros((MT, T))
        for c, (k, m) in enumerate(chan):
            clean = rS[c] + gN * rN[c]
            u = urand(stream_key(sd, ST_SELF, k, m), T)
            g = 10 ** (-(selfnoiseSNR - 10 * np.log10(np.mean(clean ** 2) / np.mean(u ** 2))) / 20)
            sn[c] = g * u
            data[s, c] = clean + sn[c]
            cs[s, c] = rS[c]
        for c, (k, m) in enumerate(chan):
            cn[s, c] = gN * rN[c] + sn[base[k]]
    return data, cs, cn, vad
