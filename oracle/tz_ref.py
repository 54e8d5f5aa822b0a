"""TEST INFRASTRUCTURE ONLY -- float64 CPU restatement of the reference's
time-domain (T(z)) few-samples compression, SURVEY §8a row a14:
``dist_fct_approx`` (``danse_toolbox/d_base.py:1941-1991``),
``extract_few_samples_from_convolution`` (``d_base.py:1538-1566``) and
``danse_compression_few_samples`` (``d_base.py:1871-1938``).  Pinned against
the reference's own functions on seeded inputs (``tests/golden/tz_*.npz``).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla

from .danse_ref_cpu import back_to_time_domain


def dist_fct_approx(wHat, h, f, R):
    """``d_base.py:1941-1991``: (2n-1)-tap IR of the WOLA filtering with the
    frequency-domain filters wHat [n/2+1 x M] (diagonal sums of
    diag(f) circulant(flip(w_td)) diag(h)), divided by R."""
    n = len(h)
    wTD = back_to_time_domain(wHat.conj(), n, axis=0)
    wTD = np.real(wTD)
    out = np.zeros((2 * n - 1, wTD.shape[1]))
    for m in range(wTD.shape[1]):
        Hmat = sla.circulant(np.flip(wTD[:, m]))
        Amat = np.diag(f) @ Hmat @ np.diag(h)
        for ii in range(-n + 1, n):
            out[ii + n - 1, m] = np.trace(Amat, ii)
    return out / R


def dist_fct_approx_closed(wHat, h, f, R):
    """Closed form of the same IR: wIR[tau + n - 1] = c[(-tau) mod n] *
    sum_i f[i] h[i + tau] / R with c = flip(w_td) (the trace of the offset
    diagonal of diag(f) C diag(h), C circulant)."""
    n = len(h)
    wTD = np.real(back_to_time_domain(wHat.conj(), n, axis=0))
    c = np.flip(wTD, axis=0)
    taus = np.arange(-n + 1, n)
    S = np.correlate(h, f, 'full')          # S[tau + n - 1] = sum_i f[i] h[i + tau]
    return (c[(-taus) % n, :] * S[:, None]) / R


def extract_few_samples_from_convolution(idDesired, a, b):
    """``d_base.py:1538-1566``."""
    out = np.zeros(len(idDesired))
    yqzp = np.concatenate((np.zeros(len(a)), b, np.zeros(len(a))))
    for ii in range(len(idDesired)):
        out[ii] = np.dot(yqzp[idDesired[ii] + 1:idDesired[ii] + 1 + len(a)], np.flip(a))
    return out


def danse_compression_few_samples(yq, wqqHat, L, wIRprevious, h, f, Ns, updateBroadcastFilter=False):
    """``d_base.py:1871-1938``: the last L samples of the T(z)-filtered
    local frame, summed over the node's sensors."""
    wIR = dist_fct_approx(wqqHat, h, f, Ns) if updateBroadcastFilter else wIRprevious
    y = np.zeros((L, yq.shape[-1]))
    for m in range(yq.shape[-1]):
        idDesired = np.arange(start=len(wIR) - L + 1, stop=len(wIR) + 1)
        y[:, m] = extract_few_samples_from_convolution(idDesired, wIR[:, m], yq[:, m])
    return np.sum(y, axis=1), wIR
