"""Where does the fp32 device error of large-D online DANSE come from?

Runs the float64 oracle (test infrastructure) with single-precision rounding
injected at one stage at a time and reports the per-bin filter error against
the pure float64 run (after gating), as the GPU parity tests measure it:

  fft32    : WOLA analysis spectra computed in single precision
  scm32    : SCMs rounded to complex64 after every recursion step
  solve32  : GEVD / MWF solved in complex64 (LAPACK chegvd)
  state32  : fft32 + scm32, solve in float64  (an fp64 solve on fp32 state)
  all32    : everything single precision (the all-fp32 device design)

Usage: python scripts/precision_probe.py [case] [mode ...]
"""
from __future__ import annotations

import sys
from multiprocessing import Pool
from pathlib import Path

import numpy as np
import scipy.fft as sfft
import scipy.linalg as sla

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tests'))
sys.path.insert(0, str(ROOT / 'tests' / 'golden'))

from oracle import danse_ref_cpu as O  # noqa: E402
from golden_cases import ONLINE_CASES, BATTERY  # noqa: E402
from _util import make_case_params, make_case_scene  # noqa: E402

CASES = {
    'C19': dict(name='C19', M=[4] * 16, dur=4.0, seed=21, danse=dict(ONLINE_CASES[1]['danse'], nodeUpdating='asy')),
    'B11': dict(name='B11', M=[4] * 8, dur=4.0, seed=31, danse=dict(BATTERY, nodeUpdating='asy')),
    'D39s': dict(name='D39s', M=[8] * 32, dur=4.0, seed=41, danse=dict(BATTERY, nodeUpdating='seq')),
}


def gevd32(Ryy, Rnn, refSensorIdx, rank=1):
    out = np.zeros((Ryy.shape[0], Ryy.shape[-1]), dtype=complex)
    for f in range(Ryy.shape[0]):
        s, X = sla.eigh(Ryy[f].astype(np.complex64), Rnn[f].astype(np.complex64))
        idx = np.flip(np.argsort(s))
        s, X = s[idx], X[:, idx]
        Q = np.linalg.inv(X.conj().T)
        D = np.zeros(len(s), dtype=np.float32)
        D[:rank] = 1 - 1 / s[:rank]
        out[f] = ((X * D) @ Q.conj().T)[:, refSensorIdx]
    return out


def gevd_mix(Ryy, Rnn, refSensorIdx, rank=1, rq64=False):
    """fp64 Cholesky + zhegst, C rounded to complex64 for the eigen step
    (complex64 LAPACK eigh), fp64 back-transform x = L^-H v."""
    out = np.zeros((Ryy.shape[0], Ryy.shape[-1]), dtype=complex)
    for f in range(Ryy.shape[0]):
        L = np.linalg.cholesky(Rnn[f])
        Li = sla.solve_triangular(L, np.eye(L.shape[0]), lower=True)
        C = Li @ Ryy[f] @ Li.conj().T
        s, V = np.linalg.eigh(C.astype(np.complex64))
        idx = np.flip(np.argsort(s))
        s, V = s[idx].astype(np.float64), V[:, idx].astype(np.complex128)
        g = L.conj().T[:, refSensorIdx]
        for r in range(rank):
            v = V[:, r] / np.linalg.norm(V[:, r])
            lam = np.real(v.conj() @ C @ v) if rq64 else s[r]
            x = sla.solve_triangular(L.conj().T, v, lower=False)
            out[f] += (1 - 1 / lam) * x * (v.conj() @ g)
    return out


def gevd_planD(Ryy, Rnn, refSensorIdx, rank=1):
    """planC with the triangular inverse in float32: fp64 Cholesky of Rnn,
    L rounded to complex64, Li = L^-1 by complex64 substitution, then the
    planC float32 congruence / eigen / back-transform."""
    out = np.zeros((Ryy.shape[0], Ryy.shape[-1]), dtype=complex)
    for f in range(Ryy.shape[0]):
        L = np.linalg.cholesky(Rnn[f]).astype(np.complex64)
        Li = sla.solve_triangular(L, np.eye(L.shape[0], dtype=np.complex64), lower=True).astype(np.complex64)
        A32 = Ryy[f].astype(np.complex64)
        C = Li @ A32 @ Li.conj().T
        s, V = np.linalg.eigh(C)
        idx = np.flip(np.argsort(s))
        s, V = s[idx], V[:, idx]
        g = L.conj().T[:, refSensorIdx]
        for r in range(rank):
            v = V[:, r]
            x = Li.conj().T @ v
            out[f] += (1 - 1 / float(s[r])) * x * complex(v.conj() @ g)
    return out


def gevd_planA(Ryy, Rnn, refSensorIdx, rank=1, li32=False, cong32=False):
    """The device plan: Ryy as stored (fp32), fp64 Cholesky of Rnn, fp64
    triangular inverse, C = Linv Ryy Linv^H in fp64 rounded to complex64,
    complex64 eigen step, x = Linv^H v in fp64."""
    out = np.zeros((Ryy.shape[0], Ryy.shape[-1]), dtype=complex)
    for f in range(Ryy.shape[0]):
        L = np.linalg.cholesky(Rnn[f])
        Li = sla.solve_triangular(L, np.eye(L.shape[0]), lower=True)
        if cong32:
            L32, A32 = Li.astype(np.complex64), Ryy[f].astype(np.complex64)
            C = L32 @ A32 @ L32.conj().T
        else:
            C = (Li @ Ryy[f] @ Li.conj().T).astype(np.complex64)
        s, V = np.linalg.eigh(C)
        idx = np.flip(np.argsort(s))
        s, V = s[idx], V[:, idx]
        g = L.conj().T[:, refSensorIdx].astype(np.complex64)
        for r in range(rank):
            v = V[:, r]
            x = (Li.astype(np.complex64).conj().T @ v) if li32 else (Li.conj().T @ v.astype(complex))
            out[f] += (1 - 1 / float(s[r])) * x * complex(v.conj() @ g)
    return out


def run(args):
    cname, mode = args
    case = CASES[cname]
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    fft32 = mode in ('fft32', 'state32', 'all32', 'mixC', 'mixD', 'ryy32', 'rnn32', 'planA', 'planB', 'planC', 'planD')
    ryyAcc32 = mode in ('planA', 'planB', 'planC', 'planD')
    scm32 = mode in ('scm32', 'state32', 'all32')
    solve32 = mode in ('solve32', 'all32')

    class Probe(O.OnlineDANSE):
        def _fft(self, y):
            if not fft32:
                return super()._fft(y)
            x = (y * self.h[:, None]).astype(np.float32)
            return (sfft.fft(x, self.N, axis=0)[:self.F, :] / np.float32(np.sqrt(self.Ns))).astype(np.complex128)

        def _scm_update(self, k, s, y, vad):
            super()._scm_update(k, s, y, vad)
            if scm32 or ryyAcc32:
                s.Ryy = s.Ryy.astype(np.complex64).astype(np.complex128)
            if scm32:
                s.Rnn = s.Rnn.astype(np.complex64).astype(np.complex128)

    saved = O.update_w_gevd
    if solve32:
        O.update_w_gevd = gevd32
    elif mode == 'planA':
        O.update_w_gevd = gevd_planA
    elif mode == 'planC':
        O.update_w_gevd = lambda a, b, refSensorIdx, rank=1: gevd_planA(a, b, refSensorIdx, rank, li32=True, cong32=True)
    elif mode == 'planD':
        O.update_w_gevd = gevd_planD
    elif mode == 'planB':
        O.update_w_gevd = lambda a, b, refSensorIdx, rank=1: gevd_planA(a, b, refSensorIdx, rank, li32=True)
    elif mode == 'ryy32':
        O.update_w_gevd = lambda a, b, refSensorIdx, rank=1: gevd_mix(a.astype(np.complex64).astype(complex), b, refSensorIdx, rank)
    elif mode == 'rnn32':
        O.update_w_gevd = lambda a, b, refSensorIdx, rank=1: gevd_mix(a, b.astype(np.complex64).astype(complex), refSensorIdx, rank)
    elif mode in ('mixC', 'mixD'):
        O.update_w_gevd = lambda a, b, refSensorIdx, rank=1: gevd_mix(a, b, refSensorIdx, rank, rq64=(mode == 'mixD'))
    try:
        ov = Probe(sc, dp, vadMinProp=wp.vadMinProportionActive).run()
    finally:
        O.update_w_gevd = saved
    return cname, mode, [w.copy() for w in ov.wTilde], ov.startRound.copy(), ov.d.copy()


def main():
    cname = sys.argv[1] if len(sys.argv) > 1 else 'C19'
    modes = sys.argv[2:] or ['fp64', 'fft32', 'scm32', 'solve32', 'state32', 'all32']
    if 'fp64' not in modes:
        modes = ['fp64'] + modes
    with Pool(len(modes)) as pool:
        res = pool.map(run, [(cname, m) for m in modes])
    base = res[0]
    K = len(base[2])
    for _, mode, w, st, d in res[1:]:
        errs, per_t = [], []
        for k in range(K):
            s0 = int(base[3][k])
            a, b = w[k][:, s0 + 1:], base[2][k][:, s0 + 1:]
            e = np.linalg.norm(a - b, axis=-1) / np.maximum(np.linalg.norm(b, axis=-1), 1e-30)
            errs.append(e.ravel())
            p99t = np.percentile(e, 99, axis=0)
            per_t.append((p99t[:10].mean(), p99t[-20:].mean()))
        e = np.concatenate(errs)
        pt = np.mean(np.array(per_t), axis=0)
        de = np.max(np.abs(d - base[4])) / np.max(np.abs(base[4]))
        print(f'{cname} {mode:8s} median {np.median(e):.2e} p99 {np.percentile(e, 99):.2e} max {e.max():.2e} '
              f'| d {de:.2e} | p99 first10 {pt[0]:.2e} last20 {pt[1]:.2e}', flush=True)


if __name__ == '__main__':
    main()
