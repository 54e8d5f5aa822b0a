"""TEST INFRASTRUCTURE ONLY — float64 CPU restatement of the reference DANSE
engine (online + batch, fully connected).  Used as the parity checker for the
HIP path and as bench.py's ``cpu_baseline`` ("port").  Never imported by the
product package ``danse_amd``.

Each function names the reference code it restates (``/root/reference``
paths).  Arithmetic is done with the same NumPy/SciPy calls, in the same
order, so that results match the reference to ~1e-12 (checked against golden
vectors produced by the reference itself: ``tests/test_oracle_golden.py``).
Differences from the reference are storage-only: no per-frame ỹ / yyᴴ /
centralised-SCM history (the reference's O(nIter) allocations,
``d_classes.py:726-777``), only the current frame.

Supported: seq / asy / sim node updating, MWF and rank-R GEVD updates,
``use1stFrameAsBasis``, SCM init types, filter init types, wholeChunk
broadcasts, local / centralised / single-sensor-broadcast estimates,
pre-given filters (the SNR replay), Oracle-SRO phase compensation with
full-sample-drift flags, and the batch engine (``d_batch.py``).
"""
from __future__ import annotations

import copy
import types

import numpy as np
import scipy.linalg as sla
import scipy.signal as sig

from danse_amd.scheduler import initialize_events

from ._gevd_pool import eigh_bins, gevd_w_bins, set_workers  # noqa: F401


# --------------------------------------------------------------------------- #
# Helpers (d_base.py)
# --------------------------------------------------------------------------- #

def init_complex_filter(size, refIdx=0, initType='selectFirstSensor', fixedValue=0., seed=0):
    """``d_base.py:2367-2414``."""
    if initType == 'selectFirstSensor':
        w = np.zeros(size, dtype=complex)
        if len(size) == 3:
            w[:, :, refIdx] = 1
        elif len(size) == 2:
            w[:, refIdx] = 1
    elif initType == 'random':
        rng = np.random.default_rng(seed)
        w = (rng.random(size) - 0.5) + 1j * (rng.random(size) - 0.5)
    elif initType == 'fixedValue':
        w = np.full(size, fill_value=fixedValue, dtype=complex)
    elif initType == 'selectFirstSensor_andFixedValue':
        w = np.full(size, fill_value=fixedValue, dtype=complex)
        if len(size) == 3:
            w[:, :, refIdx] = 1
        elif len(size) == 2:
            w[:, refIdx] = 1
    else:
        raise ValueError(initType)
    return w


def init_covmats(dims, rng, covMatInitType, covMatRandomInitScaling, covMatEyeInitScaling):
    """``d_base.py:2417-2470``."""
    randArray = 2 * rng.random(dims) - 1 + 1j * (2 * rng.random(dims) - 1)
    if covMatInitType == 'fully_random':
        return covMatRandomInitScaling * randArray
    eye = np.eye(dims[-1]) * covMatEyeInitScaling
    if len(dims) == 3:
        eye = np.tile(eye, (dims[0], 1, 1))
    if covMatInitType == 'eye_and_random':
        return eye + covMatRandomInitScaling * randArray
    if covMatInitType == 'eye':
        return eye
    raise ValueError(covMatInitType)


def back_to_time_domain(x, n, axis=0):
    """``d_base.py:1482-1535``; like the reference it forces DC/Nyquist real
    IN PLACE in the caller's array (quirk Q7)."""
    flagSingleton = False
    if x.ndim == 1:
        x = x[:, np.newaxis]
        flagSingleton = True
    if axis == 1:
        x = x.T
    if x.shape[0] != n / 2 + 1:
        raise ValueError('`x` should be (n/2+1)-long along the IFFT axis.')
    x[0, :] = x[0, :].real
    x[-1, :] = x[-1, :].real
    x = np.concatenate((x, np.flip(x[:-1, :].conj(), axis=0)[:-1, :]), axis=0)
    if flagSingleton:
        x = np.squeeze(x)
    xout = np.fft.ifft(x, n, axis=0)
    if axis == 1:
        xout = xout.T
    return xout


def local_chunk(y, idxEnd, N):
    """``local_chunk_for_broadcast`` / ``local_chunk_for_update``
    (``d_base.py:1391-1479``) given the integer frame end."""
    idxBeg = max(idxEnd - N, 0)
    chunk = y[idxBeg:idxEnd, :]
    if idxEnd - idxBeg < N:
        chunk = np.concatenate((np.zeros((N - chunk.shape[0], chunk.shape[1])), chunk))
    return chunk, idxBeg, idxEnd


def compression_whole_chunk(yq, wHat, h, f, zqPrevious, Ns):
    """``danse_compression_whole_chunk`` (``d_base.py:1759-1868``)."""
    N = len(yq)
    if wHat.shape[-1] == 1:
        wHat1 = np.squeeze(wHat)
        yqHat = np.fft.fft(np.squeeze(yq) * h, N, axis=0) / np.sqrt(Ns)
        yqHat = yqHat[:N // 2 + 1]
        zqHat = wHat1.conj() * yqHat
    else:
        yqHat = np.fft.fft(np.squeeze(yq) * h[:, np.newaxis], N, axis=0) / np.sqrt(Ns)
        yqHat = yqHat[:N // 2 + 1, :]
        zqHat = np.einsum('ij,ij->i', wHat.conj(), yqHat)
    zqCurr = np.sqrt(Ns) * back_to_time_domain(zqHat, N, axis=0)
    zqCurr = np.real(zqCurr)
    zqCurr *= f
    if not np.any(zqPrevious):
        zq = zqCurr
    else:
        zq = np.zeros(N)
        zq[:(N - Ns)] = zqPrevious[-(N - Ns):]
        zq += zqCurr
        nOverlaps = N // Ns
        normVal = np.zeros(N + Ns)
        for ii in range(nOverlaps):
            normVal[ii * Ns:ii * Ns + N] += h ** 2
        normVal = normVal[Ns:]
        zq[:Ns] /= normVal[:Ns]
    return zqHat, zq


def desired_sig_chunk(w, y, win, normFactWOLA, dChunk):
    """``get_desired_sig_chunk`` 'wola' branch (``d_base.py:2027-2084``);
    ``dChunk`` is a view of ``d`` and is updated in place."""
    dhatCurr = np.einsum('ij,ij->i', w.conj(), y)
    dChunkCurr = normFactWOLA * win * back_to_time_domain(dhatCurr, len(win))
    if len(dChunk) < len(win):
        dChunk += np.real(dChunkCurr[-len(dChunk):])
    else:
        dChunk += np.real(dChunkCurr)
    return dChunk, dhatCurr


def get_stft(x, fs, win, ovlp, boundary=None):
    """``d_base.py:2284-2338``."""
    if x.ndim == 1:
        x = x[:, np.newaxis]
    for c in range(x.shape[-1]):
        _, _, tmp = sig.stft(x[:, c], fs=fs, window=win, nperseg=len(win),
                             noverlap=int(ovlp * len(win)), return_onesided=True, boundary=boundary)
        if c == 0:
            out = np.zeros((tmp.shape[0], tmp.shape[1], x.shape[-1]), dtype=complex)
        out[:, :, c] = tmp
    return out


def get_istft(x, fs, win, ovlp, boundary=None):
    """``d_base.py:2341-2364`` (single channel)."""
    _, out = sig.istft(x, fs=fs, window=win, nperseg=len(win), noverlap=int(ovlp * len(win)), boundary=boundary)
    return out


# --------------------------------------------------------------------------- #
# Filter updates (d_classes.py:3320-3387)
# --------------------------------------------------------------------------- #

def update_w(Ryy, Rnn, refSensorIdx, rank=None):
    """MWF update, ``d_classes.py:3320-3340``."""
    Evect = np.zeros(Ryy.shape[-1])
    Evect[refSensorIdx] = 1
    ryd = np.matmul(Ryy - Rnn, Evect)
    Ryyinv = np.linalg.inv(Ryy)
    w = np.matmul(Ryyinv, ryd[:, :, np.newaxis])
    return w[:, :, 0]


def update_w_gevd(Ryy, Rnn, refSensorIdx, rank=1):
    """Rank-R GEVD update, ``d_classes.py:3343-3387`` (per-bin
    ``scipy.linalg.eigh(Ryy, Rnn)``, descending sort, W = X D X^{-1})."""
    n = Ryy.shape[-1]
    nFreqs = Ryy.shape[0]
    # with worker processes (oracle/_gevd_pool.py) the whole per-bin
    # computation below runs in them, chunked over bins (bit-identical)
    wp = gevd_w_bins(Ryy, Rnn, refSensorIdx, rank)
    if wp is not None:
        return wp
    Xmat = np.zeros((nFreqs, n, n), dtype=complex)
    sigma = np.zeros((nFreqs, n))
    # the per-bin eigh calls (serial, or spread over worker processes with
    # bit-identical results: oracle/_gevd_pool.py)
    S, Xall = eigh_bins(Ryy, Rnn)
    for kappa in range(nFreqs):
        s, X = S[kappa], Xall[kappa]
        idx = np.flip(np.argsort(s))
        sigma[kappa, :] = s[idx]
        Xmat[kappa] = X[:, idx]
    Qmat = np.linalg.inv(np.transpose(Xmat.conj(), axes=[0, 2, 1]))
    Dmat = np.zeros((nFreqs, n, n))
    for r in range(rank):
        Dmat[:, r, r] = np.squeeze(1 - 1 / sigma[:, r])
    Qh = np.transpose(Qmat.conj(), axes=[0, 2, 1])
    fullW = np.matmul(np.matmul(Xmat, Dmat), Qh)
    return fullW[:, :, refSensorIdx]


def update_w_gevd_refs(Ryy, Rnn, refs, rank=1):
    """``update_w_gevd`` for several reference indices on the same SCMs (the
    centralised filters of every node, ``d_batch.py:95-104``): the full
    ``X D Q^H`` product is computed once and its columns picked, so each
    result is bit-identical to a separate ``update_w_gevd`` call."""
    n = Ryy.shape[-1]
    nFreqs = Ryy.shape[0]
    Xmat = np.zeros((nFreqs, n, n), dtype=complex)
    sigma = np.zeros((nFreqs, n))
    S, Xall = eigh_bins(Ryy, Rnn)
    for kappa in range(nFreqs):
        s, X = S[kappa], Xall[kappa]
        idx = np.flip(np.argsort(s))
        sigma[kappa, :] = s[idx]
        Xmat[kappa] = X[:, idx]
    Qmat = np.linalg.inv(np.transpose(Xmat.conj(), axes=[0, 2, 1]))
    Dmat = np.zeros((nFreqs, n, n))
    for r in range(rank):
        Dmat[:, r, r] = np.squeeze(1 - 1 / sigma[:, r])
    Qh = np.transpose(Qmat.conj(), axes=[0, 2, 1])
    fullW = np.matmul(np.matmul(Xmat, Dmat), Qh)
    return [fullW[:, :, r] for r in refs]


def update_w_refs(Ryy, Rnn, refs, rank=None):
    """``update_w`` for several reference indices (one inverse, bit-identical
    per reference to separate calls)."""
    Ryyinv = np.linalg.inv(Ryy)
    out = []
    for r in refs:
        Evect = np.zeros(Ryy.shape[-1])
        Evect[r] = 1
        ryd = np.matmul(Ryy - Rnn, Evect)
        out.append(np.matmul(Ryyinv, ryd[:, :, np.newaxis])[:, :, 0])
    return out


def update_covmats_batch(yAllFrames, vadAllFrames):
    """``d_classes.py:3272-3304``."""
    if len(vadAllFrames) > yAllFrames.shape[1]:
        vadAllFrames = vadAllFrames[:yAllFrames.shape[1]]
    v = vadAllFrames.astype(bool)
    # the reference's mean over frames of einsum('ikj,ikl->ikjl') outer
    # products, as one matmul per bin (the einsum materialises F x T x D x D:
    # 7.8 GB per node at config D's D = 39)

    def mean_outer(Y):
        return np.matmul(np.swapaxes(Y, 1, 2), Y.conj()) / Y.shape[1]
    return mean_outer(yAllFrames[:, v, :]), mean_outer(yAllFrames[:, ~v, :])


def cohdrift_sro_estimation_ls(wPos, wPri, avgResProd, Ns, ld, alpha, first, bufferFlagPos, bufferFlagPri):
    """``cohdrift_sro_estimation`` with ``method='ls'`` (``d_sros.py:19-95``)."""
    res = wPos * wPri.conj()
    res = np.concatenate([res[:-1], np.conj(res)[::-1][:-1]], -1)
    res *= np.exp(1j * 2 * np.pi / len(res) * np.arange(len(res)) * (bufferFlagPos - bufferFlagPri))
    avg = res if first else alpha * avgResProd + (1 - alpha) * res
    kappa = np.arange(0, len(wPri))
    b = np.pi * kappa * (ld * Ns) / (len(kappa) * 2)
    sro = - b.T @ np.angle(avg[-len(kappa):]) / (b.T @ b)
    return sro, avg


def _is_hermitian_and_posdef(x):
    x = np.real_if_close(x)
    b1 = np.allclose(np.transpose(x, axes=(0, 2, 1)).conj(), x)
    b2 = True
    for ii in range(x.shape[0]):
        if any(np.linalg.eigvalsh(x[ii]) < 0):
            b2 = False
            break
    return b1 and b2


def _full_rank(mat):
    return (np.linalg.matrix_rank(mat) == mat.shape[-1]).all()


def scm_gate(Rnn, Ryy, gevd):
    """``check_covariance_matrices`` helpers (``d_classes.py:1447-1480``)."""
    if gevd:
        return (_is_hermitian_and_posdef(Rnn) and _is_hermitian_and_posdef(Ryy)
                and _full_rank(Rnn) and _full_rank(Ryy))
    return _full_rank(Rnn) and _full_rank(Ryy)


def vad_per_frame(vad, frameLen, frameShift, minProp):
    """``WASN.get_vad_per_frame`` (``siggen/classes.py:669-702``)."""
    n = len(vad)
    out = np.zeros(n // frameShift)
    for ii in range(len(out)):
        b, e = ii * frameShift, ii * frameShift + frameLen
        if e > n:
            out = out[:ii + 1]
            break
        chunk = vad[b:e]
        out[ii] = float(sum(chunk) >= len(chunk) * minProp)
    return out.astype(bool)


def beta_from_t50p(t50p, fs, Ns):
    """``prep_for_danse._get_beta_from_t50p`` (``d_core.py:485-503``)."""
    return np.exp(np.log(0.5) / (t50p * fs / Ns))


# --------------------------------------------------------------------------- #
# Online engine (DANSEvariables, d_classes.py:370-2709)
# --------------------------------------------------------------------------- #

class _SCMSet:
    """One (Ryy, Rnn, w-history, start flag) estimator family."""

    def __init__(self, Ryy, Rnn, w):
        self.Ryy = Ryy
        self.Rnn = Rnn
        self.w = w
        self.start = False


class OnlineDANSE:
    """Restatement of ``d_core.danse`` (``d_core.py:26-102``) over
    ``DANSEvariables`` (``d_classes.py:478-2709``)."""

    def __init__(self, scene, p, vadMinProp=0.5, yinOverride=None, keepHistory=True, maxRounds=None,
                 sroEstimates=None, skipDanse=False, centrBins=None, centrNodes=None):
        self.p = p
        # Test-side restrictions for the wide centralised family (sum(M) up to
        # 256), exact for synchronous wholeChunk runs, where the centralised
        # vector is the nodes' raw frames and does not depend on any filter:
        #   skipDanse   no DANSE-family SCMs, gate or solves (the broadcasts
        #               carry the initial filters; the node counters still run)
        #   centrBins   the centralised family on these bins only (its SCMs,
        #               gate and filters; dCentr / dHatCentr are not formed)
        #   centrNodes  the centralised family of these nodes only
        self.skipDanse = skipDanse
        self.centrBins = None if centrBins is None else np.asarray(centrBins, dtype=int)
        self.centrNodes = None if centrNodes is None else set(int(k) for k in centrNodes)
        self.scene = scene
        wasn = scene.wasn
        K = len(wasn)
        self.K = K
        N, Ns = p.DFTsize, p.Ns
        self.N, self.Ns = N, Ns
        self.F = N // 2 + 1
        self.M = [nd.nSensors for nd in wasn]
        self.Mtot = int(sum(self.M))
        self.neighbors = [list(nd.neighborsIdx) for nd in wasn]
        self.T = wasn[0].data.shape[0]
        self.nIter = int((self.T - N) / Ns) + 1
        self.maxRounds = maxRounds
        # estimateSROs 'DXCPPhaT' (the build's extension; the reference
        # raises, quirk Q12): the per-iteration estimates [K][nIter][K - 1]
        # come from outside (the device estimators) and take the place of the
        # Oracle values in update_sro_estimates
        self.extEst = sroEstimates
        self.seqNU = 'seq' in p.nodeUpdating
        self.h = p.winWOLAanalysis
        self.f = p.winWOLAsynthesis
        ref = p.referenceSensor
        self.ref = ref
        # inputs
        pg = p.preGivenFilters
        if yinOverride is not None:
            self.yin = yinOverride
        elif pg.active and pg.purpose == 'noise-only':
            self.yin = [nd.cleannoise for nd in wasn]
        elif pg.active and pg.purpose == 'speech-only':
            self.yin = [nd.cleanspeech for nd in wasn]
        else:
            self.yin = [nd.data for nd in wasn]
        # prep_for_danse (d_core.py:466-547)
        self.beta = []
        self.betaWext = []
        for nd in wasn:
            self.beta.append(p.forcedBeta if p.forcedBeta is not None else beta_from_t50p(p.t_expAvg50p, nd.fs, Ns))
            self.betaWext.append(p.forcedBetaExternalFilters if p.forcedBetaExternalFilters is not None
                                 else beta_from_t50p(p.t_expAvg50pExternalFilters, nd.fs, Ns))
        wasnVad = [vad_per_frame(nd.vad[:, 0] if nd.vad.ndim > 1 else nd.vad, N, Ns, vadMinProp) for nd in wasn]
        self.oVAD = wasnVad
        c = np.zeros(len(wasnVad[0]))
        for k in range(K):
            c += wasnVad[k]
        c /= K
        self.centrVAD = c.astype(bool)
        self.dimY = np.array([self.M[k] + len(self.neighbors[k]) for k in range(K)])
        self.keepHistory = keepHistory
        self._init_state()

    # ---- init_from_wasn (d_classes.py:478-985) ----
    def _init_state(self):
        p, K, F = self.p, self.K, self.F
        rng = np.random.default_rng(p.seed)
        args = (p.covMatInitType, p.covMatRandomInitScaling, p.covMatEyeInitScaling)
        if p.covMatInitType == 'batch_estimates':
            # (the reference raises here: d_classes.py:1002-1005, see danse_amd.engine.init_scm_slices)
            raise TypeError("'bool' object is not subscriptable")
        if p.covMatSameInitForAllNodes:
            dims = (self.Mtot, self.Mtot) if p.covMatSameInitForAllFreqs else (F, self.Mtot, self.Mtot)
            fullSlice = init_covmats(dims, rng, *args)
        nh = self.nIter + 1
        fi = dict(initType=p.filterInitType, fixedValue=p.filterInitFixedValue)
        self.danse, self.local, self.centr, self.ssbc = [], [], [], []
        self.wExt, self.wExtTarget = [], []
        for k in range(K):
            D = self.dimY[k]
            if not p.covMatSameInitForAllNodes:
                dims = (self.Mtot, self.Mtot) if p.covMatSameInitForAllFreqs else (F, self.Mtot, self.Mtot)
                fullSlice = init_covmats(dims, rng, *args)
            # (the reference always allocates every family's SCMs and filter
            # histories, d_classes.py:619-620 -- at K = 32 x 8 the centralised
            # ones alone are ~34 GB; the restatement builds only the enabled
            # families, which leaves every computed value unchanged)
            if p.covMatSameInitForAllFreqs:
                def tile(s):
                    return np.tile(s, (F, 1, 1))
            else:
                def tile(s):
                    return s
            ax = (slice(None),) if not p.covMatSameInitForAllFreqs else ()

            def fam(dim, on, ref=p.referenceSensor):
                if not on:
                    return _SCMSet(None, None, None)
                sl = fullSlice[ax + (slice(0, dim), slice(0, dim))]
                return _SCMSet(tile(sl), tile(sl), init_complex_filter((F, nh, dim), ref, **fi))

            refC = int(np.sum(self.M[:k]) + p.referenceSensor)
            self.danse.append(fam(D, True))
            self.ssbc.append(fam(D, p.computeSingleSensorBroadcast))
            self.wExt.append(init_complex_filter((F, nh, self.M[k]), p.referenceSensor, **fi))
            self.wExtTarget.append(init_complex_filter((F, self.M[k]), p.referenceSensor, **fi))
            cf_ = fam(self.Mtot, p.computeCentralised and (self.centrNodes is None or k in self.centrNodes), refC)
            if self.centrBins is not None and cf_.Ryy is not None:
                cf_ = _SCMSet(cf_.Ryy[self.centrBins].copy(), cf_.Rnn[self.centrBins].copy(),
                              cf_.w[self.centrBins].copy())
            self.centr.append(cf_)
            self.local.append(fam(self.M[k], p.computeLocal))
        self.i = np.zeros(K, dtype=int)
        # condition numbers (d_classes.py:965-984)
        self.condNumbers = types.SimpleNamespace(
            **{f: [np.empty((self.F, 0)) for _ in range(K)] for f in ('cn_RyyDANSE', 'cn_RyyLocal', 'cn_RyyCentr')},
            **{f: [[] for _ in range(K)] for f in ('iter_cn_RyyDANSE', 'iter_cn_RyyLocal', 'iter_cn_RyyCentr')})
        self._cnLast = [[-1] * K for _ in range(3)]
        self.numUpdatesRyy = np.zeros(K, dtype=int)
        self.numUpdatesRnn = np.zeros(K, dtype=int)
        self.d = np.zeros((self.T, K))
        self.dCentr = np.zeros_like(self.d)
        self.dLocal = np.zeros_like(self.d)
        self.dSSBC = np.zeros_like(self.d)
        self.dhat = np.zeros((F, self.nIter, K), dtype=complex)
        self.dHatCentr = np.zeros_like(self.dhat)
        self.dHatLocal = np.zeros_like(self.dhat)
        self.dHatSSBC = np.zeros_like(self.dhat)
        self.zLocal = [np.array([]) for _ in range(K)]
        self.zFullTD = [np.array([]) for _ in range(K)]
        self.zBuffer = [[np.array([]) for _ in self.neighbors[k]] for k in range(K)]
        self.z = [np.empty((self.N, 0)) for _ in range(K)]
        self.yLocalCentr = [np.array([]) for _ in range(K)]
        self.yBufferCentr = [[np.empty((0, self.M[q])) for q in range(K) if q != k] for k in range(K)]
        self.yc = [np.empty((self.N, 0)) for _ in range(K)]
        self.bufferFlags = [np.zeros((self.nIter, len(self.neighbors[k]))) for k in range(K)]
        self.bufferFlagsCentr = [np.zeros((self.nIter, K)) for _ in range(K)]
        self.phaseShiftFactors = [np.zeros(self.dimY[k]) for k in range(K)]
        self.phaseShiftFactorsCentr = [np.zeros(self.Mtot) for _ in range(K)]
        self.SROsppm = np.array([nd.sro for nd in self.scene.wasn])
        self.SROsEstimates = [np.zeros((self.nIter, len(self.neighbors[k]))) for k in range(K)]
        self.SROsResiduals = [np.zeros((self.nIter, len(self.neighbors[k]))) for k in range(K)]
        # CohDrift (d_classes.py:2364-2470, d_sros.py:19-95): per-iteration
        # coherences yyH[0, q] / sqrt(yyH[0, 0] yyH[q, q]) and the averaged
        # residual products (2 (F - 1) bins, the reference's full-spectrum layout)
        self.cohHist = [np.zeros((self.nIter, self.F, len(self.neighbors[k])), dtype=complex) for k in range(K)]
        self.avgProdResiduals = [np.zeros((2 * (self.F - 1), len(self.neighbors[k])), dtype=complex)
                                 for k in range(K)]
        self.nInternalFilterUps = np.zeros(K)
        self.lastExtFiltUp = np.zeros(K)
        self.nSensorsNeighborsCentr = [[self.M[q] for q in range(K) if q != k] for k in range(K)]
        self.startRound = np.full(K, -1)
        self.startRoundCentr = np.full(K, -1)
        # fewSamples broadcasting state (d_classes.py:522, 658-663, 828-831):
        # T(z) IR initialised as a Dirac at tap N (not N - 1) on the reference sensor
        self.lastBroadcastInstant = np.zeros(K)
        self.lastTDfilterUp = np.zeros(K)
        self.timeInstants = np.stack([nd.timeStamps for nd in self.scene.wasn], axis=1)
        self.wIR = []
        for k in range(K):
            wt = np.zeros((2 * self.N - 1, self.M[k]))
            wt[self.N, p.referenceSensor] = 1
            self.wIR.append(wt)

    # ---- driver (d_core.py:66-90) ----
    def run(self):
        p = self.p
        ts = [nd.timeStamps for nd in self.scene.wasn]
        nodeFs = [nd.fs for nd in self.scene.wasn]
        events, fs = initialize_events(ts, nodeFs, p, self.neighbors)
        self.events, self.fsEv = events, fs
        nUp = 0
        import time as _time
        self.roundTimes = [(int(np.min(self.i)), _time.perf_counter())]
        # (progressEvery: a progress line on stderr every that many rounds --
        # long parity runs on the GPU box must keep writing)
        pe = getattr(self, 'progressEvery', None)
        lastRep = 0
        for ev in events:
            for ii in range(ev.nEvents):
                k = ev.nodes[ii]
                if ev.type[ii] == 'bc':
                    self.broadcast(ev.t, fs[k], k)
                elif ev.type[ii] == 'up':
                    if self.maxRounds is not None and self.i[k] >= self.maxRounds:
                        continue
                    self.update_and_estimate(ev.t, fs[k], k, ev.bypassUpdate[ii])
                    nUp += 1
            self.roundTimes.append((int(np.min(self.i)), _time.perf_counter()))
            if pe and self.roundTimes[-1][0] >= lastRep + pe:
                lastRep = self.roundTimes[-1][0]
                import sys as _sys
                print(f'# oracle round {lastRep} ({self.roundTimes[-1][1] - self.roundTimes[0][1]:.1f} s)',
                      file=_sys.stderr, flush=True)
            if self.maxRounds is not None and np.all(self.i >= self.maxRounds):
                break
        self.nUpdateEvents = nUp
        return self

    # ---- broadcast (d_classes.py:1043-1128) ----
    def broadcast(self, tCurr, fs, k):
        p = self.p
        idxEnd = int(np.floor(tCurr * fs))
        ykFrame, _, _ = local_chunk(self.yin[k], idxEnd, self.N)
        if p.computeCentralised:
            # pre_fill_buffers_centralised (d_classes.py:1162-1183)
            if p.broadcastType == 'wholeChunk':
                self.yLocalCentr[k] = ykFrame
            elif p.efficientSpSBC:
                self.yLocalCentr[k] = ykFrame[-self._bc_size(k, tCurr):, :]
            else:
                raise NotImplementedError('centralised fewSamples without efficientSpSBC (reference raises too)')
        if p.broadcastType == 'wholeChunk':
            _, self.zLocal[k] = compression_whole_chunk(
                ykFrame, self.wExt[k][:, self.i[k], :], self.h, self.f, self.zLocal[k], self.Ns)
            self.zFullTD[k] = np.concatenate((self.zFullTD[k], self.zLocal[k][:self.Ns]))
            chunk = self.zLocal[k][:self.Ns]
            n = self.Ns
        elif p.broadcastType == 'fewSamples':
            # d_classes.py:1090-1125: IR refresh every upTDfilterEvery seconds,
            # currL = L floor(samples since last broadcast / L) (efficientSpSBC)
            from . import tz_ref
            upd = False
            if np.abs(tCurr - self.lastTDfilterUp[k]) >= p.upTDfilterEvery:
                if not (p.noFusionAtSingleSensorNodes and self.M[k] == 1):
                    upd = True
                self.lastTDfilterUp[k] = tCurr
            if p.efficientSpSBC:
                currL = self._bc_size(k, tCurr)
                self.lastBroadcastInstant[k] = tCurr
            else:
                currL = int(p.broadcastLength)
            self.zLocal[k], self.wIR[k] = tz_ref.danse_compression_few_samples(
                ykFrame, self.wExt[k][:, self.i[k], :], currL, self.wIR[k], self.h, self.f, self.Ns,
                updateBroadcastFilter=upd)
            n = -currL
            chunk = self.zLocal[k][n:] if currL > 0 else np.array([])
        else:
            raise ValueError(p.broadcastType)
        # fill_buffers / fill_buffers_centr (d_classes.py:1185-1250)
        for q in self.neighbors[k]:
            idx = self.neighbors[q].index(k)
            self.zBuffer[q][idx] = np.concatenate((self.zBuffer[q][idx], chunk), axis=0)
        if p.computeCentralised:
            if n > 0:
                ych = self.yLocalCentr[k][:n, :]
            elif n < 0:
                ych = self.yLocalCentr[k][n:, :]
            else:
                ych = np.empty((0, self.M[k]))
            for q in range(self.K):
                if q != k and self._centr_on(q):
                    idx = k if k < q else k - 1
                    self.yBufferCentr[q][idx] = np.concatenate((self.yBufferCentr[q][idx], ych), axis=0)

    def _bc_size(self, k, tCurr):
        """``get_buffer_size_for_efficient_bc`` (d_classes.py:1130-1160)."""
        L_ = int(self.p.broadcastLength)
        n = np.sum((self.timeInstants[:, k] > self.lastBroadcastInstant[k]) & (self.timeInstants[:, k] <= tCurr))
        return int(L_ * np.floor(n / L_))

    # ---- process_incoming_signals_buffers (d_classes.py:1701-1807) ----
    def _process_buffers(self, k):
        N, Ns = self.N, self.Ns
        zk = np.empty((N, 0))
        flags = np.zeros(len(self.neighbors[k]))
        for iq in range(len(self.neighbors[k])):
            buf = self.zBuffer[k][iq]
            Bq = len(buf)
            if self.i[k] == 0:
                if Bq == N:
                    cur = buf
                elif Bq < N:
                    flags[iq] = -1 * int(abs(N - Bq))
                    cur = np.concatenate((np.zeros(N - Bq), buf), axis=0)
                else:
                    flags[iq] = +1 * int(abs(N - Bq))
                    cur = buf[-N:]
            else:
                if Bq < Ns:
                    flags[iq] = -1 * int(abs(Ns - Bq))
                elif Bq > Ns:
                    flags[iq] = +1 * int(abs(Ns - Bq))
                if N - Bq > 0:
                    cur = np.concatenate((self.z[k][-(N - Bq):, iq], buf), axis=0)
                else:
                    cur = buf
            zk = np.concatenate((zk, cur[:, np.newaxis]), axis=1)
        self.z[k] = zk
        self.bufferFlags[k][self.i[k], :] = flags
        self.zBuffer[k] = [np.array([]) for _ in self.neighbors[k]]
        if self._centr_on(k):
            self._process_buffers_centr(k)

    def _process_buffers_centr(self, k):
        N, Ns, K = self.N, self.Ns, self.K
        yk = np.empty((N, 0))
        flags = np.zeros(K)
        for q in range(K):
            if q == k:
                continue
            iq = q - 1 if q > k else q
            buf = self.yBufferCentr[k][iq]
            Bq = len(buf)
            if self.i[k] == 0:
                if Bq == N:
                    cur = buf
                elif Bq < N:
                    cur = np.concatenate((np.zeros((N - Bq, buf.shape[-1])), buf), axis=0)
                    flags[q] = -1 * int(abs(N - Bq))
                else:
                    cur = buf[-N:, :]
                    flags[q] = +1 * int(abs(N - Bq))
            else:
                if Bq < Ns:
                    flags[q] = -1 * int(abs(Ns - Bq))
                elif Bq > Ns:
                    flags[q] = +1 * int(abs(Ns - Bq))
                if N - Bq > 0:
                    if iq == 0:
                        s = 0
                    else:
                        s = int(np.sum([self.M[ii] for ii in range(K) if ii != k and ii < q]))
                    e = s + self.M[q]
                    cur = np.concatenate((self.yc[k][-(N - Bq):, s:e], buf), axis=0)
                else:
                    cur = buf
            yk = np.concatenate((yk, cur), axis=1)
        self.yc[k] = yk
        self.bufferFlagsCentr[k][self.i[k], :] = flags
        self.yBufferCentr[k] = [np.empty((0, self.M[q])) for q in range(K) if q != k]

    def _fft(self, y):
        return (np.fft.fft(y * self.h[:, np.newaxis], self.N, axis=0) / np.sqrt(self.Ns))[:self.F, :]

    def _centr_on(self, k):
        return self.p.computeCentralised and (self.centrNodes is None or k in self.centrNodes)

    def _cbins(self, yHat):
        return yHat if self.centrBins is None else yHat[self.centrBins]

    # ---- update_and_estimate (d_classes.py:1252-1330) ----
    def update_and_estimate(self, tCurr, fs, k, bypass):
        p = self.p
        N, Ns = self.N, self.Ns
        i = self.i[k]
        if k == p.referenceSensor and self.nInternalFilterUps[k] == 0:
            self.firstDANSEupdateRefSensor = tCurr
        self._process_buffers(k)
        # local_chunk_for_update (d_base.py:1427-1479): WOLA lag N - Ns for wholeChunk only
        idxEnd = int(np.floor(tCurr * fs)) - ((N - Ns) if p.broadcastType == 'wholeChunk' else 0)
        yLoc, self.idxBeg, self.idxEnd = local_chunk(self.yin[k], idxEnd, N)
        # build_ytilde (1893-1934)
        yT = np.concatenate((yLoc, self.z[k]), axis=1)
        yTHat = self._fft(yT)
        if self._centr_on(k):
            cols = []
            cov = 0
            for q in range(self.K):
                if q == k:
                    cols.append(yLoc)
                else:
                    b = int(np.sum(self.nSensorsNeighborsCentr[k][:cov]))
                    e = int(np.sum(self.nSensorsNeighborsCentr[k][:cov + 1]))
                    cols.append(self.yc[k][:, b:e])
                    cov += 1
            yC = np.concatenate([np.empty((N, 0))] + cols, axis=1)
            yCHat = self._fft(yC)
        if p.computeSingleSensorBroadcast:
            cols = [copy.deepcopy(yLoc)]
            cov = 0
            for q in range(self.K):
                if q != k:
                    b = int(np.sum(self.nSensorsNeighborsCentr[k][:cov]))
                    cols.append(self.yc[k][:, b][:, np.newaxis])
                    cov += 1
            yS = np.concatenate(cols, axis=1)
            ySHat = self._fft(yS)
        yLHat = yTHat[:, :self.M[k]].copy() if p.computeLocal else None
        # compensate_sros (1936-2046)
        skipUpdate = False
        extra = np.zeros(self.dimY[k])
        for q in range(len(self.neighbors[k])):
            fl = self.bufferFlags[k][i, q]
            if not np.isnan(fl):
                extra[self.M[k] + q] = fl
            else:
                skipUpdate = True
        yUncomp = yTHat.copy()
        if p.compensateSROs:
            if p.includeFSDflags:
                self.phaseShiftFactors[k] += extra
            psf = np.exp(-1 * 1j * 2 * np.pi / N * np.outer(np.arange(self.F), self.phaseShiftFactors[k]))
            yTHat *= psf
        if p.estimateSROs == 'CohDrift':
            yc = yTHat if p.cohDrift.loop == 'closed' else yUncomp
            D = yc.shape[1]
            for q in range(len(self.neighbors[k])):
                iq = self.M[k] + q
                yy0q = yc[:, 0] * yc[:, iq].conj() / D
                yy00 = yc[:, 0] * yc[:, 0].conj() / D
                yyqq = yc[:, iq] * yc[:, iq].conj() / D
                self.cohHist[k][i, :, q] = yy0q / np.sqrt(yy00 * yyqq)
        skipUpdateCentr = None
        if self._centr_on(k):
            skipUpdateCentr = False
            extraC = np.zeros(self.Mtot)
            for q in range(self.K):
                if q != k:
                    fl = self.bufferFlagsCentr[k][i, q]
                    if not np.isnan(fl):
                        b = int(np.sum(self.nSensorsNeighborsCentr[k][:q]))
                        e = int(np.sum(self.nSensorsNeighborsCentr[k][:(q + 1)]))
                        if e == b:
                            e += 1
                        extraC[b:e] = fl
                    else:
                        skipUpdateCentr = True
            if p.compensateSROs:
                if p.includeFSDflags:
                    self.phaseShiftFactorsCentr[k] += extraC
                psfC = np.exp(-1 * 1j * 2 * np.pi / N * np.outer(np.arange(self.F), self.phaseShiftFactorsCentr[k]))
                yCHat *= psfC
        if p.computeSingleSensorBroadcast and p.compensateSROs:
            raise NotImplementedError('SRO compensation for single-sensor broadcast not implemented yet.')

        if p.preGivenFilters.active:
            pg = p.preGivenFilters
            self.danse[k].w[:, i + 1, :] = pg.internalFilters[k][:, i + 1, :]
            self.wExt[k][:, i + 1, :] = pg.externalFilters[k][:, i + 1, :]
            if p.computeLocal:
                self.local[k].w[:, i + 1, :] = pg.filtersLocal[k][:, i + 1, :]
            if self._centr_on(k):
                self.centr[k].w[:, i + 1, :] = self._cbins(pg.filtersCentr[k][:, i + 1, :])
            if p.computeSingleSensorBroadcast:
                self.ssbc[k].w[:, i + 1, :] = pg.filtersSSBC[k][:, i + 1, :]
        else:
            vad = self.oVAD[k][i]
            if vad:
                self.numUpdatesRyy[k] += 1
            else:
                self.numUpdatesRnn[k] += 1
            if not self.skipDanse:
                self._scm_update(k, self.danse[k], yTHat, vad)
            if p.computeLocal:
                self._scm_update(k, self.local[k], yLHat, vad)
            if self._centr_on(k):
                self._scm_update(k, self.centr[k], self._cbins(yCHat), self.centrVAD[i])
            if p.computeSingleSensorBroadcast:
                self._scm_update(k, self.ssbc[k], ySHat, vad)
            self._cond_numbers(k, i)
            self._check_covmats(k, tCurr)
            if not skipUpdate and not bypass:
                self._perform_update(k, skipUpdateCentr)
            else:
                self.danse[k].w[:, i + 1, :] = self.danse[k].w[:, i, :]
                if p.computeLocal:
                    self.local[k].w[:, i + 1, :] = self.local[k].w[:, i, :]
                if bypass:
                    if self._centr_on(k):
                        self.centr[k].w[:, i + 1, :] = self.centr[k].w[:, i, :]
                    if p.computeSingleSensorBroadcast:
                        self.ssbc[k].w[:, i + 1, :] = self.ssbc[k].w[:, i, :]
            self._update_external_filters(k, tCurr)
        # update_sro_estimates (Oracle only) + phase shifts (2364-2621)
        if p.estimateSROs == 'Oracle':
            sroOut = (self.SROsppm[self.neighbors[k]] - self.SROsppm[k]) * 1e-6
            self.SROsResiduals[k][i, :] = sroOut
        elif p.estimateSROs == 'CohDrift':
            if self.extEst is not None:
                # replay: the residual estimates of another run (the device's)
                # drive the same closed-loop accumulation (a test of the loop
                # against the estimator, tests/test_gpu_engine_modes.py)
                self.SROsResiduals[k][i, :] = self.extEst[k][i, :]
            else:
                self._cohdrift(k, i)
        elif p.estimateSROs == 'DXCPPhaT':
            self.SROsResiduals[k][i, :] = self.extEst[k][i, :]
        if p.compensateSROs:
            for q in range(len(self.neighbors[k])):
                if p.estimateSROs == 'DXCPPhaT':
                    self.SROsEstimates[k][i, q] = self.extEst[k][i, q]
                elif p.estimateSROs == 'CohDrift':
                    res = self.SROsResiduals[k][i, q]
                    if p.cohDrift.loop == 'closed':
                        self.SROsEstimates[k][i, q] += res / (1 + res) * p.cohDrift.alphaEps
                    else:
                        self.SROsEstimates[k][i, q] = res / (1 + res)
                else:
                    self.SROsEstimates[k][i, q] = (self.SROsppm[self.neighbors[k][q]] - self.SROsppm[k]) * 1e-6
                self.phaseShiftFactors[k][self.M[k] + q] -= self.SROsEstimates[k][i, q] * self.Ns
            if p.computeCentralised:
                for q in range(self.K):
                    est = (self.SROsppm[q] - self.SROsppm[k]) * 1e-6
                    b = int(np.sum(self.M[:q]))
                    e = int(np.sum(self.M[:q + 1]))
                    self.phaseShiftFactorsCentr[k][b:e] -= est * self.Ns
        # get_desired_signal (2623-2709)
        if p.desSigProcessingType == 'conv':
            self._conv_estimates(k, i, yT, yC if p.computeCentralised else None, yLoc,
                                 yS if p.computeSingleSensorBroadcast else None)
            self.i[k] += 1
            return
        nf = np.sqrt(self.Ns)
        sl = slice(self.idxBeg, self.idxEnd)
        _, dh = desired_sig_chunk(self.danse[k].w[:, i + 1, :], yTHat, self.f, nf, self.d[sl, k])
        self.dhat[:, i, k] = dh
        if self._centr_on(k) and self.centrBins is None:
            _, dh = desired_sig_chunk(self.centr[k].w[:, i + 1, :], yCHat, self.f, nf, self.dCentr[sl, k])
            self.dHatCentr[:, i, k] = dh
        if p.computeLocal:
            _, dh = desired_sig_chunk(self.local[k].w[:, i + 1, :], yLHat, self.f, nf, self.dLocal[sl, k])
            self.dHatLocal[:, i, k] = dh
        if p.computeSingleSensorBroadcast:
            _, dh = desired_sig_chunk(self.ssbc[k].w[:, i + 1, :], ySHat, self.f, nf, self.dSSBC[sl, k])
            self.dHatSSBC[:, i, k] = dh
        self.i[k] += 1

    # ---- get_desired_signal with desSigProcessingType 'conv'
    # (get_desired_sig_chunk, d_base.py:2085-2100; d_classes.py:2623-2709):
    # per family, wIR = dist_fct_approx(w[:, i+1, :], win_s, win_s, Ns) (the
    # closed form, oracle/tz_ref.py, equal to the reference's diagonal sums to
    # ~1e-16), the last Ns samples (idDesired = len - Ns .. len - 1) of the
    # convolutions of its first M_k columns with the first M_k channels of
    # the family's time-domain update frame, summed, into d[idxEnd - Ns,
    # idxEnd); dhat is None (NaN in the complex array) ----
    def _conv_estimates(self, k, i, yT, yC, yLoc, yS):
        from . import tz_ref
        p, Ns, Mk = self.p, self.Ns, self.M[k]
        sl = slice(self.idxEnd - Ns, self.idxEnd)

        def chunk(w, yTD):
            wIR = tz_ref.dist_fct_approx_closed(w, self.f, self.f, Ns)
            idD = np.arange(start=len(wIR) - Ns, stop=len(wIR))
            out = np.zeros((Ns, Mk))
            for m in range(Mk):
                out[:, m] = tz_ref.extract_few_samples_from_convolution(idD, wIR[:, m], yTD[:, m])
            return np.sum(out, axis=1)
        self.d[sl, k] = chunk(self.danse[k].w[:, i + 1, :], yT)
        self.dhat[:, i, k] = np.nan
        if p.computeCentralised:
            self.dCentr[sl, k] = chunk(self.centr[k].w[:, i + 1, :], yC)
            self.dHatCentr[:, i, k] = np.nan
        if p.computeLocal:
            self.dLocal[sl, k] = chunk(self.local[k].w[:, i + 1, :], yLoc)
            self.dHatLocal[:, i, k] = np.nan
        if p.computeSingleSensorBroadcast:
            self.dSSBC[sl, k] = chunk(self.ssbc[k].w[:, i + 1, :], yS)
            self.dHatSSBC[:, i, k] = np.nan

    # ---- condition numbers (d_classes.py:2126-2186, ConditionNumbers
    # .get_new_cond_number / compute_condition_numbers, d_classes.py:19-130):
    # np.linalg.cond of every bin's Ryy after the frame's update, every
    # saveConditionNumberEvery iterations, per family ----
    def _cond_numbers(self, k, i):
        p = self.p
        if not getattr(p, 'saveConditionNumber', False):
            return
        cn = self.condNumbers
        fams = [('DANSE', self.danse[k], 'cn_RyyDANSE', 'iter_cn_RyyDANSE', self._cnLast[0])]
        if p.computeLocal:
            fams.append(('local', self.local[k], 'cn_RyyLocal', 'iter_cn_RyyLocal', self._cnLast[1]))
        if self._centr_on(k):
            fams.append(('centralised', self.centr[k], 'cn_RyyCentr', 'iter_cn_RyyCentr', self._cnLast[2]))
        for _, fam, fc, fi, last in fams:
            if i - last[k] >= p.saveConditionNumberEvery:
                c = np.array([np.linalg.cond(fam.Ryy[kappa]) for kappa in range(fam.Ryy.shape[0])])
                getattr(cn, fc)[k] = np.concatenate((getattr(cn, fc)[k], c[:, np.newaxis]), axis=1)
                getattr(cn, fi)[k].append(i)
                last[k] = i

    # ---- spatial_covariance_matrix_update + conditional_scm_updating (2048-2267) ----
    def _scm_update(self, k, s: _SCMSet, y, vad):
        beta = self.beta[k]
        yyH = 1 / y.shape[1] * np.einsum('ij,ik->ijk', y, y.conj())
        # beta * R + (1 - beta) * yyH, elementwise in the same order as the
        # reference (bit-identical), without the extra temporaries
        yyH_w = (1 - beta) * yyH

        def avg(R):
            out = beta * R
            out += yyH_w
            return out
        RyyCurr, RnnCurr = s.Ryy, s.Rnn
        if vad:
            RyyCurr = avg(s.Ryy)
        else:
            RnnCurr = avg(s.Rnn)
        if self.p.use1stFrameAsBasis:
            if self.numUpdatesRyy[k] == 1 and vad:
                s.Ryy = yyH
            elif self.numUpdatesRyy[k] > 1:
                s.Ryy = RyyCurr
            if self.numUpdatesRnn[k] == 1 and not vad:
                s.Rnn = yyH
            elif self.numUpdatesRnn[k] > 1:
                s.Rnn = RnnCurr
        else:
            s.Ryy = RyyCurr
            s.Rnn = RnnCurr

    # ---- check_covariance_matrices (1430-1540) ----
    def _check_covmats(self, k, tCurr):
        p = self.p
        g = p.performGEVD
        fams = [('danse', self.danse[k], not self.skipDanse)]
        if p.simType == 'online':
            fams += [('local', self.local[k], p.computeLocal), ('centr', self.centr[k], self._centr_on(k)),
                     ('ssbc', self.ssbc[k], p.computeSingleSensorBroadcast)]
        for name, s, on in fams:
            if not on or s.start or tCurr < p.startUpdatesAfterAtLeast:
                continue
            D = s.Ryy.shape[-1]
            if self.numUpdatesRyy[k] > D and self.numUpdatesRnn[k] > D:
                if scm_gate(s.Rnn, s.Ryy, g):
                    s.start = True
                    if name == 'danse':
                        self.startRound[k] = self.i[k]
                    elif name == 'centr':
                        self.startRoundCentr[k] = self.i[k]

    # ---- perform_update (2290-2362) ----
    def _perform_update(self, k, skipUpdateCentr):
        p = self.p
        i = self.i[k]
        fn = update_w_gevd if p.performGEVD else update_w
        rank = p.GEVDrank if p.performGEVD else 1
        if p.bypassUpdates:
            return
        if self.danse[k].start:
            self.danse[k].w[:, i + 1, :] = fn(self.danse[k].Ryy, self.danse[k].Rnn, refSensorIdx=p.referenceSensor, rank=rank)
            self.nInternalFilterUps[k] += 1
        if self._centr_on(k) and self.centr[k].start and p.simType != 'batch':
            if not skipUpdateCentr:
                self.centr[k].w[:, i + 1, :] = fn(self.centr[k].Ryy, self.centr[k].Rnn,
                                                  refSensorIdx=int(np.sum(self.M[:k]) + p.referenceSensor), rank=rank)
            else:
                self.centr[k].w[:, i + 1, :] = self.centr[k].w[:, i, :]
        if p.computeLocal and self.local[k].start and p.simType != 'batch':
            self.local[k].w[:, i + 1, :] = fn(self.local[k].Ryy, self.local[k].Rnn, refSensorIdx=p.referenceSensor, rank=rank)
        if p.computeSingleSensorBroadcast and self.ssbc[k].start and p.simType != 'batch':
            self.ssbc[k].w[:, i + 1, :] = fn(self.ssbc[k].Ryy, self.ssbc[k].Rnn, refSensorIdx=p.referenceSensor, rank=rank)

    # ---- update_sro_estimates, CohDrift branch (2364-2470) ----
    def _cohdrift(self, k, i):
        p = self.p
        cd = p.cohDrift
        if p.computeCentralised:
            raise NotImplementedError('CohDrift with centralised estimates')
        if cd.estimationMethod != 'ls':
            raise NotImplementedError("CohDrift estimationMethod 'gs' (paderwasn max_time_lag_search)")
        idx = np.arange(cd.startAfterNups + cd.estEvery, self.nIter, cd.estEvery)
        if i not in idx:
            return
        first = i == np.amin(idx)
        ld = cd.segLength
        bfPos = p.broadcastLength * np.sum(self.bufferFlags[k][:(i + 1), :], axis=0)
        bfPri = p.broadcastLength * np.sum(self.bufferFlags[k][:(i - ld + 1), :], axis=0)
        if cd.loop == 'closed':
            bfPos = np.zeros_like(bfPos)
            bfPri = np.zeros_like(bfPri)
        for q in range(len(self.neighbors[k])):
            sro, apr = cohdrift_sro_estimation_ls(self.cohHist[k][i, :, q], self.cohHist[k][i - ld, :, q],
                                                  self.avgProdResiduals[k][:, q], self.Ns, ld, cd.alpha, first,
                                                  bfPos[q], bfPri[q])
            self.SROsResiduals[k][i, q] = sro
            self.avgProdResiduals[k][:, q] = apr

    # ---- update_external_filters (1627-1694) ----
    def _update_external_filters(self, k, t):
        p = self.p
        i = self.i[k]
        cur = self.danse[k].w[:, i + 1, :self.M[k]]
        if p.onlyBroadcastRefSensorSigs:
            m = np.zeros((self.wExt[k].shape[0], self.wExt[k].shape[2]), dtype=complex)
            m[:, p.referenceSensor] = 1
            self.wExt[k][:, i + 1, :] = m
        elif self.M[k] == 1 and p.noFusionAtSingleSensorNodes:
            self.wExt[k][:, i + 1, :] = self.wExt[k][:, i, :]
        elif p.noExternalFilterRelaxation or 'seq' in p.nodeUpdating:
            self.wExt[k][:, i + 1, :] = cur
        else:
            self.wExt[k][:, i + 1, :] = self.betaWext[k] * self.wExt[k][:, i, :] + \
                (1 - self.betaWext[k]) * self.wExtTarget[k]
            if t is None:
                upd = True
            else:
                upd = t - self.lastExtFiltUp[k] >= p.timeBtwExternalFiltUpdates
                if upd:
                    self.lastExtFiltUp[k] = t
            if upd:
                self.wExtTarget[k] = (1 - p.alphaExternalFilters) * self.wExtTarget[k] + p.alphaExternalFilters * cur

    # ---- outputs (the `dv` fields of SURVEY §8b) ----
    @property
    def wTilde(self):
        return [s.w for s in self.danse]

    @property
    def wTildeExt(self):
        return self.wExt

    @property
    def wLocal(self):
        return [s.w for s in self.local]

    @property
    def wCentr(self):
        return [s.w for s in self.centr]

    @property
    def wSSBC(self):
        return [s.w for s in self.ssbc]


def danse(scene, p, **kw):
    """``d_core.danse`` (``d_core.py:26-102``)."""
    return OnlineDANSE(scene, p, **kw).run()


def generate_signals_for_snr_computation(scene, p, dv, vadMinProp=0.5):
    """``d_core.py:550-599``: two replays with the recorded filters."""
    pU = copy.deepcopy(p)
    from danse_amd.params import PreComputedFilters
    pU.preGivenFilters = PreComputedFilters(
        active=True, internalFilters=dv.wTilde, externalFilters=dv.wTildeExt,
        filtersCentr=dv.wCentr, filtersSSBC=dv.wSSBC, filtersLocal=dv.wLocal, purpose='noise-only')
    dn = danse(scene, pU, vadMinProp=vadMinProp)
    pU.preGivenFilters.purpose = 'speech-only'
    ds = danse(scene, pU, vadMinProp=vadMinProp)
    return {'n': dn.d, 'n_c': dn.dCentr, 'n_l': dn.dLocal, 'n_ssbc': dn.dSSBC,
            's': ds.d, 's_c': ds.dCentr, 's_l': ds.dLocal, 's_ssbc': ds.dSSBC}


# --------------------------------------------------------------------------- #
# Batch engine (d_batch.py:3-205, d_core.py:251-352)
# --------------------------------------------------------------------------- #

class BatchDANSE:
    def __init__(self, scene, p, vadMinProp=0.5):
        self.p = p
        wasn = scene.wasn
        self.K = K = len(wasn)
        N, Ns = p.DFTsize, p.Ns
        self.N, self.Ns, self.F = N, Ns, N // 2 + 1
        self.M = [nd.nSensors for nd in wasn]
        self.neighbors = [list(nd.neighborsIdx) for nd in wasn]
        self.fs = [nd.fs for nd in wasn]
        self.yin = [nd.data for nd in wasn]
        self.clean = [nd.cleanspeech for nd in wasn]
        self.T = wasn[0].data.shape[0]
        self.nIter = int((self.T - N) / Ns) + 1
        self.win = p.winWOLAanalysis
        self.oVAD = [vad_per_frame(nd.vad[:, 0], N, Ns, vadMinProp) for nd in wasn]
        self.yinSTFT = [get_stft(self.yin[k], self.fs[k], self.win, 1 - Ns / N) * np.sum(self.win) for k in range(K)]
        fi = dict(initType=p.filterInitType, fixedValue=p.filterInitFixedValue)
        nh = p.maxBatchUpdates + 1
        self.dimY = [self.M[k] + len(self.neighbors[k]) for k in range(K)]
        self.wTilde = [init_complex_filter((self.F, max(nh, self.nIter + 1), self.dimY[k]), p.referenceSensor, **fi) for k in range(K)]
        self.wTildeExt = [init_complex_filter((self.F, max(nh, self.nIter + 1), self.M[k]), p.referenceSensor, **fi) for k in range(K)]
        self.wTildeExtTarget = [init_complex_filter((self.F, self.M[k]), p.referenceSensor, **fi) for k in range(K)]
        self.betaWext = [p.forcedBetaExternalFilters if p.forcedBetaExternalFilters is not None
                         else beta_from_t50p(p.t_expAvg50pExternalFilters, self.fs[k], Ns) for k in range(K)]
        self.i = np.zeros(K, dtype=int)
        self.d = np.zeros((self.T, K))
        self.dhat = np.zeros((self.F, self.nIter, K), dtype=complex)
        self.mmseCost = np.full((p.maxBatchUpdates, K), None)
        self.Ryy = [None] * K
        self.Rnn = [None] * K
        self.yTildeBatch = [None] * K

    def get_y_tilde_batch(self, k):
        """``d_base.py:2473-2542`` fully connected branch (K9)."""
        zB = np.zeros((self.yinSTFT[k].shape[0], self.yinSTFT[k].shape[1], len(self.neighbors[k])), dtype=complex)
        for ii, q in enumerate(self.neighbors[k]):
            ff = self.wTildeExt[q][:, self.i[q], :]
            # einsum('ij,ikj->ik', conj(ff), Y_q) as a batched matrix-vector product
            zB[:, :, ii] = np.matmul(self.yinSTFT[q], ff.conj()[:, :, None])[:, :, 0]
        return np.concatenate((self.yinSTFT[k], zB), axis=-1)

    def batch_update_danse_covmats(self, k):
        self.yTildeBatch[k] = self.get_y_tilde_batch(k)
        self.Ryy[k], self.Rnn[k] = update_covmats_batch(self.yTildeBatch[k], self.oVAD[k])

    def perform_update(self, k):
        p = self.p
        fn = update_w_gevd if p.performGEVD else update_w
        rank = p.GEVDrank if p.performGEVD else 1
        self.wTilde[k][:, self.i[k] + 1, :] = fn(self.Ryy[k], self.Rnn[k], refSensorIdx=p.referenceSensor, rank=rank)

    def update_external_filters(self, k):
        p = self.p
        i = self.i[k]
        cur = self.wTilde[k][:, i + 1, :self.M[k]]
        if p.onlyBroadcastRefSensorSigs:
            m = np.zeros((self.F, self.M[k]), dtype=complex)
            m[:, p.referenceSensor] = 1
            self.wTildeExt[k][:, i + 1, :] = m
        elif self.M[k] == 1 and p.noFusionAtSingleSensorNodes:
            self.wTildeExt[k][:, i + 1, :] = self.wTildeExt[k][:, i, :]
        elif p.noExternalFilterRelaxation or 'seq' in p.nodeUpdating:
            self.wTildeExt[k][:, i + 1, :] = cur
        else:
            self.wTildeExt[k][:, i + 1, :] = self.betaWext[k] * self.wTildeExt[k][:, i, :] + \
                (1 - self.betaWext[k]) * self.wTildeExtTarget[k]
            self.wTildeExtTarget[k] = (1 - p.alphaExternalFilters) * self.wTildeExtTarget[k] + p.alphaExternalFilters * cur

    def batch_estimate(self, k):
        w = self.wTilde[k][:, self.i[k] + 1, :]
        self.dhat[:, :, k] = np.einsum('ik,ijk->ij', w.conj(), self.yTildeBatch[k][:, :-1, :])
        x = get_istft(self.dhat[:, :, k], self.fs[k], self.win, 1 - self.Ns / self.N) / np.sum(self.win)
        if len(x) < self.T:
            x = np.pad(x, (0, self.T - len(x)))
        self.d[:, k] = x

    def get_mmse_cost(self, k):
        tgt = self.clean[k][1000:-1000, self.p.referenceSensor]
        self.mmseCost[self.i[k], k] = np.mean(np.abs(tgt - self.d[1000:-1000, k]) ** 2)

    def run(self):
        """``d_core.danse_batch`` loop (``d_core.py:286-326``)."""
        p = self.p
        K = self.K
        if p.nodeUpdating == 'seq':
            up = 0
            for _ in range(p.maxBatchUpdates):
                for k in range(K):
                    self.batch_update_danse_covmats(k)
                for k in range(K):
                    if k == up:
                        self.perform_update(k)
                    else:
                        self.wTilde[k][:, self.i[k] + 1, :] = self.wTilde[k][:, self.i[k], :]
                        self.wTildeExt[k][:, self.i[k] + 1, :] = self.wTildeExt[k][:, self.i[k], :]
                    self.update_external_filters(k)
                    self.batch_estimate(k)
                    self.get_mmse_cost(k)
                    self.i[k] += 1
                up = (up + 1) % K
        else:
            for _ in range(p.maxBatchUpdates):
                for k in range(K):
                    self.batch_update_danse_covmats(k)
                for k in range(K):
                    self.perform_update(k)
                    self.update_external_filters(k)
                    self.batch_estimate(k)
                    self.get_mmse_cost(k)
                    self.i[k] += 1
        return self


def danse_batch(scene, p, vadMinProp=0.5):
    b = BatchDANSE(scene, p, vadMinProp=vadMinProp)
    # d_core.danse_batch computes the centralised / local estimates first
    # (d_core.py:282-283; no iterations for those)
    if p.computeCentralised or p.computeLocal:
        batch_family_estimates(b, centr=p.computeCentralised, local=p.computeLocal)
    return b.run()


def _centr_setup(b):
    """Centralised frame VAD and STFT (init_from_wasn, d_classes.py:905-964):
    the per-frame VAD averaged over nodes (active if any node is), the
    node-stacked STFT yCentrBatch, and the batch SCMs over it."""
    K = b.K
    v = np.zeros(len(b.oVAD[0]))
    for k in range(K):
        v += b.oVAD[k]
    v /= K
    b.centrVAD = v.astype(bool)
    b.yCentrBatch = np.concatenate(tuple(b.yinSTFT), axis=2)
    b.Ryycentr, b.Rnncentr = update_covmats_batch(b.yCentrBatch, b.centrVAD)


def batch_family_estimates(b, centr=True, local=True):
    """``get_centralized_and_local_estimates`` (``d_batch.py:20-88``): one
    filter per node from the batch SCMs of the centralised (all sensors,
    centralised VAD, reference index sum(M[:k]) + ref) and local observation
    vectors, stored in history slot i[k] + 1; estimates over all frames but
    the last, ISTFT / sum(win), and the untrimmed MMSE costs."""
    p = b.p
    fn = update_w_gevd if p.performGEVD else update_w
    rank = p.GEVDrank if p.performGEVD else 1
    fi = dict(initType=p.filterInitType, fixedValue=p.filterInitFixedValue)
    K, F, Mt = b.K, b.F, int(sum(b.M))
    _centr_setup(b)
    b.wCentr = [init_complex_filter((F, b.nIter + 1, Mt), int(np.sum(b.M[:k]) + p.referenceSensor), **fi)
                for k in range(K)]
    b.wLocal = [init_complex_filter((F, b.nIter + 1, b.M[k]), p.referenceSensor, **fi) for k in range(K)]
    b.dCentr = np.zeros((b.T, K))
    b.dLocal = np.zeros((b.T, K))
    b.dHatCentr = np.zeros((F, b.nIter, K), dtype=complex)
    b.dHatLocal = np.zeros((F, b.nIter, K), dtype=complex)

    def istft(x, k):
        y = get_istft(x, b.fs[k], b.win, 1 - b.Ns / b.N) / np.sum(b.win)
        return np.pad(y, (0, b.T - len(y))) if len(y) < b.T else y
    if centr:
        for k in range(K):
            i = b.i[k]
            b.wCentr[k][:, i + 1, :] = fn(b.Ryycentr, b.Rnncentr,
                                          refSensorIdx=int(np.sum(b.M[:k]) + p.referenceSensor), rank=rank)
            b.dHatCentr[:, :, k] = np.einsum('ik,ijk->ij', b.wCentr[k][:, i + 1, :].conj(), b.yCentrBatch[:, :-1, :])
            b.dCentr[:, k] = istft(b.dHatCentr[:, :, k], k)
    if local:
        for k in range(K):
            i = b.i[k]
            Ry, Rn = update_covmats_batch(b.yinSTFT[k], b.oVAD[k])
            b.wLocal[k][:, i + 1, :] = fn(Ry, Rn, refSensorIdx=p.referenceSensor, rank=rank)
            b.dHatLocal[:, :, k] = np.einsum('ik,ijk->ij', b.wLocal[k][:, i + 1, :].conj(), b.yinSTFT[k][:, :-1, :])
            b.dLocal[:, k] = istft(b.dHatLocal[:, :, k], k)
    b.mmseCostLocal = [np.mean(np.abs(b.clean[k][:, p.referenceSensor] - b.dLocal[:, k]) ** 2) for k in range(K)]
    b.mmseCostCentr = [np.mean(np.abs(b.clean[k][:, p.referenceSensor] - b.dCentr[:, k]) ** 2) for k in range(K)]
    return b


def get_best_perf(scene, p, wCentr=None, vadMinProp=0.5):
    """``d_core.get_best_perf`` (``d_core.py:602-627``) for fully connected
    WASNs: batch centralised estimates without SROs
    (``init_from_wasn_for_best_perf``, ``d_classes.py:378-470``: the noSRO
    signals -- here the scene signals, which carry no resampling -- or the
    noise-only / speech-only ones with pre-given filters;
    ``get_centralized_estimates``, ``d_batch.py:90-125``).  ``wCentr``: the
    filters of an earlier call (slot 1 is used).  Returns an object with
    ``wCentr``, ``dCentr``, ``dHatCentr``, ``mmseCostCentr``."""
    b = BatchDANSE(scene, p, vadMinProp=vadMinProp)
    pg = p.preGivenFilters
    if pg.active and pg.purpose == 'noise-only':
        b.yin = [nd.cleannoise for nd in scene.wasn]
    elif pg.active and pg.purpose == 'speech-only':
        b.yin = [nd.cleanspeech for nd in scene.wasn]
    b.yinSTFT = [get_stft(b.yin[k], b.fs[k], b.win, 1 - b.Ns / b.N) * np.sum(b.win) for k in range(b.K)]
    rank = p.GEVDrank if p.performGEVD else 1
    fi = dict(initType=p.filterInitType, fixedValue=p.filterInitFixedValue)
    K, F, Mt = b.K, b.F, int(sum(b.M))
    _centr_setup(b)
    b.wCentr = [init_complex_filter((F, b.nIter + 1, Mt), int(np.sum(b.M[:k]) + p.referenceSensor), **fi)
                for k in range(K)]
    b.dCentr = np.zeros((b.T, K))
    b.dHatCentr = np.zeros((F, b.nIter, K), dtype=complex)
    nseg = b.yCentrBatch.shape[1]
    idx = np.arange(nseg) if nseg == b.nIter else np.arange(nseg - 1)
    if wCentr is None:
        # (every node's call sees the same SCMs: one decomposition, the
        # references' columns -- bit-identical to K separate calls of fn)
        fnR = update_w_gevd_refs if p.performGEVD else update_w_refs
        wK = fnR(b.Ryycentr, b.Rnncentr, [int(np.sum(b.M[:k]) + p.referenceSensor) for k in range(K)], rank=rank)
    for k in range(K):
        i = b.i[k]
        if wCentr is None:
            b.wCentr[k][:, i + 1, :] = wK[k]
        else:
            b.wCentr[k][:, i + 1, :] = wCentr[k][:, i + 1, :]
        b.dHatCentr[:, :, k] = np.einsum('ik,ijk->ij', b.wCentr[k][:, i + 1, :].conj(), b.yCentrBatch[:, idx, :])
        y = get_istft(b.dHatCentr[:, :, k], b.fs[k], b.win, 1 - b.Ns / b.N) / np.sum(b.win)
        b.dCentr[:, k] = np.pad(y, (0, b.T - len(y))) if len(y) < b.T else y
    b.mmseCostCentr = [np.mean(np.abs(b.clean[k][:, p.referenceSensor] - b.dCentr[:, k]) ** 2) for k in range(K)]
    return b
