"""TEST INFRASTRUCTURE ONLY -- the oracle's per-bin generalized eigenproblems
(``scipy.linalg.eigh(Ryy[kappa], Rnn[kappa])``, ``d_classes.py:3358-3371``)
spread over worker processes.

Every bin still goes through the same ``scipy.linalg.eigh`` call on the same
matrices, so the results are bit-identical to the serial loop (checked by
``tests/test_oracle_golden.py::test_gevd_pool_bit_identical``); only the wall
time changes.  Off by default: ``bench.py``'s CPU baseline times the serial
reference path.  The heavy parity tests (config C's K = 16 x 4 with DXCP, the
north-star K = 32 x 8, centralised estimates at large sum(M)) switch it on
with ``set_workers``.

Inputs and outputs travel through one shared-memory block ([F][n][n] Ryy,
Rnn, X and [F][n] eigenvalues); the workers are started with the 'spawn'
method (a fresh interpreter per worker, nothing of the parent's GPU state).
"""
from __future__ import annotations

import atexit
import multiprocessing as mp
import os
from multiprocessing import shared_memory

import numpy as np

_POOL = None
_W = None     # worker-side shared block


def _attach(name):
    global _W
    from threadpoolctl import threadpool_limits
    # (spawned workers share the parent's resource tracker: the block stays
    # registered once, and the parent's unlink releases it)
    _W = shared_memory.SharedMemory(name=name)
    threadpool_limits(1)


def _views(buf, F, n):
    c = F * n * n
    A = np.ndarray((F, n, n), dtype=np.complex128, buffer=buf, offset=0)
    B = np.ndarray((F, n, n), dtype=np.complex128, buffer=buf, offset=16 * c)
    X = np.ndarray((F, n, n), dtype=np.complex128, buffer=buf, offset=32 * c)
    S = np.ndarray((F, n), dtype=np.float64, buffer=buf, offset=48 * c)
    return A, B, X, S


def _work(args):
    import scipy.linalg as sla
    F, n, b0, b1 = args
    A, B, X, S = _views(_W.buf, F, n)
    for kappa in range(b0, b1):
        s, x = sla.eigh(A[kappa], B[kappa])
        S[kappa] = s
        X[kappa] = x
    return b1 - b0


def gevd_w_chunk(Ryy, Rnn, S, X, ref, rank):
    """w[:, :] of update_w_gevd (d_classes.py:3343-3387) for a stack of bins
    whose eigenpairs (S ascending, X) are given: descending sort, Q = inv(X^H),
    W = X D Q^H, column ref.  Every step is a per-matrix LAPACK / BLAS call, so
    a bin's result does not depend on the stack it is computed in."""
    nF, n = S.shape
    Xmat = np.zeros((nF, n, n), dtype=complex)
    sigma = np.zeros((nF, n))
    for kappa in range(nF):
        idx = np.flip(np.argsort(S[kappa]))
        sigma[kappa, :] = S[kappa][idx]
        Xmat[kappa] = X[kappa][:, idx]
    Qmat = np.linalg.inv(np.transpose(Xmat.conj(), axes=[0, 2, 1]))
    Dmat = np.zeros((nF, n, n))
    for r in range(rank):
        Dmat[:, r, r] = np.squeeze(1 - 1 / sigma[:, r])
    Qh = np.transpose(Qmat.conj(), axes=[0, 2, 1])
    fullW = np.matmul(np.matmul(Xmat, Dmat), Qh)
    return fullW[:, :, ref]


def _work_w(args):
    import scipy.linalg as sla
    F, n, b0, b1, ref, rank = args
    A, B, X, S = _views(_W.buf, F, n)
    for kappa in range(b0, b1):
        S[kappa], X[kappa] = sla.eigh(A[kappa], B[kappa])
    w = gevd_w_chunk(A[b0:b1], B[b0:b1], S[b0:b1], X[b0:b1], ref, rank)
    X[b0:b1, 0, :] = w      # (the chunk's eigenvectors are no longer needed)
    return b1 - b0


class _Pool:
    def __init__(self, workers):
        self.workers = workers
        self.shm = None
        self.pool = None

    def _ensure(self, nbytes):
        if self.shm is not None and self.shm.size >= nbytes:
            return
        self.close()
        self.shm = shared_memory.SharedMemory(create=True, size=max(nbytes, 1 << 20))
        ctx = mp.get_context('spawn')
        # single-threaded BLAS / LAPACK in the workers from their start (the
        # environment a spawned interpreter inherits: threadpoolctl alone did
        # not hold every BLAS the workers load to one thread, and 16 workers x
        # 16 BLAS threads oversubscribed the GPU box's CPU share)
        keys = ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS', 'BLIS_NUM_THREADS')
        old = {k: os.environ.get(k) for k in keys}
        try:
            for k in keys:
                os.environ[k] = '1'
            self.pool = ctx.Pool(self.workers, initializer=_attach, initargs=(self.shm.name,))
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    def eigh(self, Ryy, Rnn):
        F, n, _ = Ryy.shape
        self._ensure(F * n * (48 * n + 8))
        A, B, X, S = _views(self.shm.buf, F, n)
        A[:] = Ryy
        B[:] = Rnn
        step = -(-F // (4 * self.workers))
        done = sum(self.pool.map(_work, [(F, n, b, min(b + step, F)) for b in range(0, F, step)]))
        assert done == F
        return S.copy(), X.copy()

    def gevd_w(self, Ryy, Rnn, ref, rank):
        F, n, _ = Ryy.shape
        self._ensure(F * n * (48 * n + 8))
        A, B, X, S = _views(self.shm.buf, F, n)
        A[:] = Ryy
        B[:] = Rnn
        step = -(-F // (4 * self.workers))
        done = sum(self.pool.map(_work_w, [(F, n, b, min(b + step, F), ref, rank) for b in range(0, F, step)]))
        assert done == F
        return X[:, 0, :].copy()

    def close(self):
        if self.pool is not None:
            self.pool.terminate()
            self.pool.join()
            self.pool = None
        if self.shm is not None:
            self.shm.close()
            self.shm.unlink()
            self.shm = None


def set_workers(n):
    """n > 1: spread the per-bin eigh calls over n worker processes; 0 or 1:
    the serial loop."""
    global _POOL
    if _POOL is not None and (n <= 1 or n != _POOL.workers):
        _POOL.close()
        _POOL = None
    if n > 1 and _POOL is None:
        _POOL = _Pool(int(n))


def eigh_bins(Ryy, Rnn):
    """(eigenvalues [F][n] ascending, eigenvectors [F][n][n]) of every bin's
    generalized problem, one ``scipy.linalg.eigh(Ryy[f], Rnn[f])`` per bin."""
    if _POOL is not None and Ryy.shape[0] >= 8:
        return _POOL.eigh(np.ascontiguousarray(Ryy, dtype=np.complex128),
                          np.ascontiguousarray(Rnn, dtype=np.complex128))
    import scipy.linalg as sla
    F, n, _ = Ryy.shape
    S = np.empty((F, n))
    X = np.empty((F, n, n), dtype=complex)
    for kappa in range(F):
        S[kappa], X[kappa] = sla.eigh(Ryy[kappa], Rnn[kappa])
    return S, X


def gevd_w_bins(Ryy, Rnn, ref, rank):
    """update_w_gevd's filters w [F][n]: with workers, each worker runs the
    whole per-bin computation (eigh, sort, inverse, product) for its chunk of
    bins; None without workers (the caller's serial path)."""
    if _POOL is not None and Ryy.shape[0] >= 8:
        return _POOL.gevd_w(np.ascontiguousarray(Ryy, dtype=np.complex128),
                            np.ascontiguousarray(Rnn, dtype=np.complex128), ref, rank)
    return None


@atexit.register
def _shutdown():
    set_workers(0)
