"""Host driver of the MI355X DANSE engine (device path only — no CPU fallback).

Turns the reference's parameters + a batch of S same-shape scenes into the
C-ABI configuration (``include/danse_mi355x.h``): integer round tables from
the host scheduler, per-(round, scene, family, node) control bytes, initial
filters / SCM slices, and device inputs held in torch tensors.  Outputs come
back in the reference's layout (the ``dv`` fields consumed by
``format_output`` / ``DANSEoutputs.from_variables``,
``danse_toolbox/d_core.py:105-127``, ``danse_toolbox/d_post.py:41-133``).

Control-byte derivation restates, per round i and node k:
  * counters ``numUpdatesRyy/Rnn`` (``d_classes.py:2094-2100``) and the
    first-frame-basis rule (``conditional_scm_updating``, 2203-2267), incl.
    quirk Q11 (centralised SCM: centralised VAD, node counters);
  * the start gate ``numUpdates > D`` (``check_covariance_matrices``,
    1482-1540); the Hermitian/PSD/rank checks are evaluated on the device
    (non-positive Cholesky pivot -> DIAG bit) instead of in fp64 on the host;
  * seq bypass from the event matrix (``build_events_matrix``,
    ``d_base.py:1160-1187``) and the external-filter timer
    (``update_external_filters``, ``d_classes.py:1680-1694``).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .scheduler import (initialize_events, compile_rounds, compile_rounds_fs, FS_BCEND, FS_LEN, FS_POS, FS_ZEND,
                        FS_IRSRC, FS_FIELDS, FS_STEP_UPDATE)
from .outputs import host_fields, stft_frames


def beta_from_t50p(t50p, fs, Ns):
    """``prep_for_danse._get_beta_from_t50p`` (``d_core.py:485-503``)."""
    return np.exp(np.log(0.5) / (t50p * fs / Ns))


def init_complex_filter(size, refIdx, initType, fixedValue):
    """``init_complex_filter`` (``d_base.py:2367-2414``).  ``random`` draws
    with the reference's default seed 0 over the whole ``size`` (the caller
    passes the reference's ``(F, nIter + 1, D)`` so the first iteration's
    slice holds the same numbers)."""
    if initType == 'selectFirstSensor':
        w = np.zeros(size, dtype=np.complex128)
        w[..., refIdx] = 1
    elif initType == 'random':
        rng = np.random.default_rng(0)
        w = (rng.random(size) - 0.5) + 1j * (rng.random(size) - 0.5)
    elif initType == 'fixedValue':
        w = np.full(size, fixedValue, dtype=np.complex128)
    elif initType == 'selectFirstSensor_andFixedValue':
        w = np.full(size, fixedValue, dtype=np.complex128)
        w[..., refIdx] = 1
    else:
        raise ValueError(f'filterInitType {initType!r}')
    return w


def init_filter_history(F, nIter, D, refIdx, initType, fixedValue):
    """Initial filter history ``(F, nIter + 1, D)`` of one family-node
    (``init_from_wasn``, ``d_classes.py:392-410,660-700``); deterministic
    init types broadcast one ``(F, D)`` slice (no copy)."""
    if initType == 'random':
        return init_complex_filter((F, nIter + 1, D), refIdx, initType, fixedValue)
    return np.broadcast_to(init_complex_filter((F, D), refIdx, initType, fixedValue)[:, None, :], (F, nIter + 1, D))


def init_scm_slices(p, Mtot, K, F):
    """``init_covmats`` (``d_base.py:2417-2470``) in the draw order of
    ``init_from_wasn`` (``d_classes.py:553-651``): one ``fullSlice`` for all
    nodes or one per node (drawn node by node from the same generator), each
    ``(Mtot, Mtot)`` or per bin ``(F, Mtot, Mtot)``.  Returns the K slices."""
    if p.covMatInitType == 'batch_estimates':
        # the reference's own error: init_covmats_from_batch calls
        # get_y_tilde_batch(k, False), whose useThisFilter=False is then
        # indexed (d_classes.py:1002-1005 -> d_base.py:2526-2528); the run
        # never starts (tests/golden/ref_modes.npz records it)
        raise TypeError("'bool' object is not subscriptable (covMatInitType 'batch_estimates': "
                        "init_covmats_from_batch, d_classes.py:1002-1005)")
    rng = np.random.default_rng(p.seed)
    dims = (Mtot, Mtot) if p.covMatSameInitForAllFreqs else (F, Mtot, Mtot)

    def draw():
        rand = 2 * rng.random(dims) - 1 + 1j * (2 * rng.random(dims) - 1)
        if p.covMatInitType == 'fully_random':
            return p.covMatRandomInitScaling * rand
        eye = np.eye(Mtot) * p.covMatEyeInitScaling
        if p.covMatInitType == 'eye_and_random':
            return eye + p.covMatRandomInitScaling * rand
        if p.covMatInitType == 'eye':
            return np.broadcast_to(eye, dims).copy()
        raise ValueError(p.covMatInitType)

    if p.covMatSameInitForAllNodes:
        one = draw()
        return [one] * K
    return [draw() for _ in range(K)]


def _cf32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.complex64)).view(np.float32)


def _ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct)) if a is not None else None


@dataclass
class FamilyInfo:
    fam: int
    name: str
    D: list       # per node
    ref: list     # per node


class DanseEngine:
    """One engine = S same-shape scenes x K nodes on one device.

    ``nodeRange`` (k0, k1) restricts the owned nodes (multi-GPU sharding);
    the fused spectra of the other nodes must then be provided between
    ``bcast`` and ``update`` (``danse_amd.dist``).
    """

    def __init__(self, scenes, p, vadMinProp=0.5, device=0, keepHistory=True, nodeRange=None,
                 pregiven=None, yin='data', yDevice=None, smallDGrid=False, resident=False):
        import torch
        self.torch = torch
        self.lib = L.load_library()
        self.p = p
        self.scenes = list(scenes)
        sc0 = self.scenes[0]
        self.S = S = len(self.scenes)
        self.K = K = sc0.nNodes
        self.M = [n.nSensors for n in sc0.wasn]
        self.Mtot = int(sum(self.M))
        self.N, self.Ns = p.DFTsize, p.Ns
        self.F = self.N // 2 + 1
        # the scene signals may live on the device only (yDevice, e.g.
        # scene.make_scenes_device): the length comes from the time stamps
        self.T = len(sc0.wasn[0].timeStamps)
        for sc in self.scenes:
            if sc.nNodes != K or [n.nSensors for n in sc.wasn] != self.M or len(sc.wasn[0].timeStamps) != self.T:
                raise ValueError('all scenes of one engine must share the WASN shape')
            if any(not np.array_equal(n.timeStamps, m.timeStamps) for n, m in zip(sc.wasn, sc0.wasn)):
                raise ValueError('all scenes of one engine must share the node clocks')
        if p.simType != 'online':
            raise ValueError('DanseEngine runs the online engine (simType online)')
        if p.desSigProcessingType not in ('wola', 'conv'):
            raise ValueError(f'desSigProcessingType {p.desSigProcessingType!r}')
        self.device = device
        self.keepHistory = keepHistory
        # latency layout: GEVD filter dimensions <= 12 on the 4 x 4 lane-grid
        # solver (four bins per wave) instead of one bin per lane
        self.smallDGrid = bool(smallDGrid)
        # resident engine (danse_engine_run_resident, csrc/resident.hpp): the
        # whole run in one persistent launch, SCMs resident in registers; it
        # runs on the 4 x 4 grid storage, so it implies smallDGrid
        self.resident = bool(resident)
        if self.resident:
            if pregiven is not None:
                raise ValueError('resident runs take no pre-given filters')
            if not p.performGEVD:
                raise NotImplementedError('resident runs: GEVD filters only')
            self.smallDGrid = True
        self.k0, self.k1 = nodeRange if nodeRange is not None else (0, K)
        self.nIter = int((self.T - self.N) / self.Ns) + 1
        neighbors = [list(n.neighborsIdx) for n in sc0.wasn]
        for k in range(K):
            if sorted(neighbors[k]) != [q for q in range(K) if q != k]:
                raise NotImplementedError('device path covers fully connected WASNs')
        events, fs = initialize_events([n.timeStamps for n in sc0.wasn], [n.fs for n in sc0.wasn], p, neighbors)
        self.events, self.fsEv = events, fs
        self.fewSamples = p.broadcastType == 'fewSamples'
        if self.fewSamples:
            self.rt = compile_rounds_fs(events, fs, p, K, [n.timeStamps for n in sc0.wasn], self.M)
        else:
            self.rt = compile_rounds(events, fs, p, K)
        self.R = R = self.rt.nRounds
        # (node-sharded engines: a fewSamples round whose updates run as
        # several node-subset steps is driven segment by segment, one exchange
        # of the late z frames before each (update_segments / update(r, seg));
        # with centralised / SSBC families the broadcast phase also analyses
        # the raw local frames of the nodes the engine does not own, which
        # their observation vectors read (BcastArgs.foreign))
        if p.computeSingleSensorBroadcast and p.compensateSROs:
            # compensate_sros raises here too (d_classes.py:2042-2044)
            raise NotImplementedError('SRO compensation for single-sensor broadcast not implemented yet.')
        self._build_sro_tables(sc0)
        self._build_centr_tables(sc0)
        if R < 1:
            raise ValueError('signal too short for one DANSE round')
        if R > self.nIter:
            raise ValueError('more rounds than reference iterations')
        # families
        fams = [L.FAM_DANSE]
        if p.computeLocal:
            fams.append(L.FAM_LOCAL)
        if p.computeCentralised:
            fams.append(L.FAM_CENTR)
        if p.computeSingleSensorBroadcast:
            fams.append(L.FAM_SSBC)
        self.fams = fams
        self.famMask = sum(1 << f for f in fams)
        ref = p.referenceSensor
        base = np.concatenate(([0], np.cumsum(self.M)[:-1])).astype(int)
        self.base = base
        self.Dfam = {
            L.FAM_DANSE: [self.M[k] + K - 1 for k in range(K)],
            L.FAM_LOCAL: list(self.M),
            L.FAM_CENTR: [self.Mtot] * K,
            L.FAM_SSBC: [self.M[k] + K - 1 for k in range(K)],
        }
        self.refFam = {
            L.FAM_DANSE: [ref] * K, L.FAM_LOCAL: [ref] * K,
            L.FAM_CENTR: [int(base[k] + ref) for k in range(K)], L.FAM_SSBC: [ref] * K,
        }
        if p.performGEVD:
            for f in fams:
                if min(self.Dfam[f]) < p.GEVDrank:
                    raise ValueError('GEVD rank larger than a filter dimension')
        self.pregiven = pregiven
        self._ran = False
        self._gateMoved = False
        # bumped whenever the flags or the gate schedule change (callers that
        # capture their own graphs of the rounds, dist.ShardedRun, re-capture)
        self.graph_gen = 0
        self._gateSpecFailed = False
        self._gateInstalled = None
        self._build_flags()
        self._build_cfg()
        # inputs [S][Mtot][T] float32 on the device
        if yDevice is not None:
            if tuple(yDevice.shape) != (S, self.Mtot, self.T) or yDevice.dtype != torch.float32 or not yDevice.is_cuda:
                raise ValueError('yDevice must be a float32 device tensor [S][sum M][T]')
            self.y = yDevice.contiguous()
        else:
            y = np.empty((S, self.Mtot, self.T), dtype=np.float32)
            for s, sc in enumerate(self.scenes):
                for k, nd in enumerate(sc.wasn):
                    arr = getattr(nd, yin)
                    y[s, base[k]:base[k] + self.M[k], :] = arr.T
            self.y = torch.from_numpy(y).to(f'cuda:{device}')
        L.check(self.lib.danse_engine_set_inputs(self.eng, ctypes.c_void_p(self.y.data_ptr())), self.eng)
        # condition numbers of Ryy (ConditionNumbers, d_classes.py:19-130,2126-2186)
        self.condEvery = int(p.saveConditionNumberEvery) if getattr(p, 'saveConditionNumber', False) else 0
        if self.condEvery:
            if self.resident:
                raise NotImplementedError('condition numbers on the resident engine')
            L.check(self.lib.danse_engine_set_cond(self.eng, self.condEvery), self.eng)
        if pregiven is not None:
            self._load_pregiven(pregiven)
        self._load_init_history()

    def _load_init_history(self):
        """filterInitType 'random': the whole init history (F, nIter + 1, D)
        of every family-node goes to the device, since a node that has not
        started updating uses the init slot of each iteration (INITSLOT)."""
        if self.p.filterInitType != 'random' or self.pregiven is not None:
            return
        if not self.keepHistory:
            raise NotImplementedError("filterInitType 'random' needs keepHistory=True (per-iteration init slots)")
        R = self.R
        for f in self.fams:
            for k in range(self.k0, self.k1):
                h = np.transpose(self._winit(f, k)[:, :R + 1, :], (1, 0, 2)).astype(np.complex64)
                self._put(L.OUT_W, f, k, np.broadcast_to(h[None], (self.S,) + h.shape))

    # ------------------------------------------------------------------ #
    def _build_sro_tables(self, sc0):
        """Fused-frame lags and SRO phase-compensation offsets per (round,
        node, sender), restating ``compensate_sros`` / ``update_sro_estimates``
        (``d_classes.py:1936-2046,2364-2621``) with Oracle estimates
        eps_q = (SRO_q - SRO_k) 1e-6: at update r, phi += flag (with
        ``includeFSDflags``), the frame is compensated with phi, then
        phi -= eps_q Ns."""
        p, K, R = self.p, self.K, self.R
        # fewSamples: the stream offsets of fsTab already select the frame
        self._zLag = (None if self.rt.synchronous or self.fewSamples
                      else np.ascontiguousarray(self.rt.zLag[:R], dtype=np.uint8))
        self._zPhase = None
        self.cohDrift = p.estimateSROs == 'CohDrift'
        self.dxcp = p.estimateSROs == 'DXCPPhaT'
        if self.dxcp:
            # the build's extension (the reference raises here, d_classes.py:
            # 2469-2481, quirk Q12): device DXCP-PhaT estimators per (receiver,
            # sender) feed the phase compensation (danse_cfg.dxcp)
            if self.fewSamples:
                raise NotImplementedError('DXCP-PhaT SRO estimation runs on wholeChunk broadcasts')
            if any(n.fs and abs(n.fs / (1 + n.sro * 1e-6) - 16000.0) > 1e-6 for n in sc0.wasn) or self.N != 1024 \
                    or 2048 % self.Ns:
                raise NotImplementedError('DXCP-PhaT (default parameters) needs 16 kHz, N = 1024 and Ns dividing 2048')
            # (node-sharded engines: the receivers' estimators read the other
            # ranks' senders' z streams, exchanged per round by
            # dist.ShardedRun through danse_engine_set_zchunk / _unpack_zchunk)
            if p.computeCentralised and p.compensateSROs:
                raise NotImplementedError('centralised estimates with DXCP-PhaT SRO estimation')
        elif self.cohDrift:
            cd = p.cohDrift
            if cd.loop not in ('closed', 'open') or cd.estimationMethod != 'ls':
                raise NotImplementedError("CohDrift on the device path: estimationMethod 'ls' (paderwasn's 'gs' is "
                                          "absent)")
            if self.fewSamples or p.computeCentralised:
                raise NotImplementedError('CohDrift on the device path: wholeChunk broadcasts, no centralised family')
            self._cdFlagWin = None
            if cd.loop == 'open':
                # bufferFlagPos - bufferFlagPri (update_sro_estimates,
                # d_classes.py:2376-2386): broadcastLength x the flags of the
                # last segLength rounds, per (round, receiver, sender)
                fl = np.asarray(self.rt.flags[:R], dtype=np.float64)
                if not np.all(np.isfinite(fl)):
                    raise NotImplementedError('CohDrift open loop with undefined (NaN) buffer flags')
                cum = np.cumsum(fl, axis=0)
                ld = int(cd.segLength)
                win = cum.copy()
                win[ld:] -= cum[:-ld]
                self._cdFlagWin = np.ascontiguousarray(float(p.broadcastLength) * win)
        elif p.estimateSROs != 'Oracle':
            raise ValueError(f'estimateSROs={p.estimateSROs!r}')
        if not p.compensateSROs:
            return
        sro = np.array([nd.sro for nd in sc0.wasn], dtype=np.float64)
        for sc in self.scenes:
            if not np.array_equal(np.array([nd.sro for nd in sc.wasn], dtype=np.float64), sro):
                raise ValueError('all scenes of one engine must share the node SROs')
        ph = np.zeros((R, K, K), dtype=np.float64)
        for k in range(K):
            phi = np.zeros(K, dtype=np.float64)
            nb = [q for q in range(K) if q != k]
            # CohDrift: the estimates accumulate on the device (cohdrift.hpp);
            # the table keeps the full-sample-drift flags only
            est = np.zeros(len(nb)) if (self.cohDrift or self.dxcp) else (sro[nb] - sro[k]) * 1e-6
            for r in range(R):
                if p.includeFSDflags:
                    phi[nb] += self.rt.flags[r, k, nb]
                ph[r, k, :] = phi
                phi[nb] -= est * self.Ns
        self._zPhase = ph

    def _build_centr_tables(self, sc0):
        """Raw-signal frames of the centralised / SSBC observation vectors
        under asynchronous clocks (``pre_fill_buffers_centralised`` /
        ``fill_buffers_centr`` / ``process_incoming_signals_buffers_centr``,
        ``d_classes.py:1162-1183,1226-1250,1809-1891``).  Every broadcast of
        sender q appends the same number of raw samples to the centralised
        buffers as to the z buffers (Ns first samples of the broadcast frame
        for wholeChunk, the last currL for fewSamples), so the buffer flags are
        the z flags and receiver k's frame of q is the last N samples of q's
        raw stream: y_q[E - N, E) with E = ``cEnd[r][q]`` (wholeChunk: the
        stream is contiguous from sample 0, checked here; fewSamples: the
        chunks' frame ends floor(t fs) can overlap or skip a sample, so the
        device keeps the raw streams themselves, danse_cfg.rawStreams), read
        with the z lag.  The
        compensation phase of the centralised vector (``compensate_sros``,
        ``d_classes.py:1996-2038``) keeps the reference's flag index
        arithmetic (quirk Q14: the flag of sender q lands on
        ``[sum(nbM[:q]), sum(nbM[:q + 1]))`` of the neighbour-size list nbM
        of node k, one channel past its end when empty) and its Oracle
        estimate index ``[sum(M[:q]), sum(M[:q + 1]))``
        (``update_sro_estimates``, ``d_classes.py:2364-2621``)."""
        p, K, R, N, Ns = self.p, self.K, self.R, self.N, self.Ns
        self._cEnd = None
        self._cPhase = None
        self._rawStreams = 0
        if self.rt.synchronous or not (p.computeCentralised or p.computeSingleSensorBroadcast):
            return
        if self.fewSamples:
            # the centralised buffers receive each chunk's raw samples into
            # per-channel streams at the z streams' positions (danse_cfg.
            # rawStreams): receiver k's frame of q ends where its z frame does
            self._rawStreams = 1
            cEnd = self.rt.fsTab[:R, :, FS_ZEND].astype(np.int64)
        else:
            bc = self.rt.bcEnd[:R]
            if R > 1 and not np.all(np.diff(bc, axis=0) == Ns):
                raise NotImplementedError('consecutive broadcast frames not Ns samples apart (raw stream gap)')
            cEnd = bc - N + Ns
        self._cEnd = np.ascontiguousarray(cEnd, dtype=np.int32)
        if not (p.compensateSROs and p.computeCentralised):
            return
        sro = np.array([nd.sro for nd in sc0.wasn], dtype=np.float64)
        M = self.M
        MT = self.Mtot
        ph = np.zeros((R, K, MT), dtype=np.float64)
        for k in range(K):
            nbM = [M[q] for q in range(K) if q != k]
            phi = np.zeros(MT, dtype=np.float64)
            for r in range(R):
                if p.includeFSDflags:
                    extra = np.zeros(MT)
                    for q in range(K):
                        if q == k:
                            continue
                        b = int(np.sum(nbM[:q]))
                        e = int(np.sum(nbM[:q + 1]))
                        if e == b:
                            e += 1
                        extra[b:e] = self.rt.flags[r, k, q]
                    phi += extra
                ph[r, k, :] = phi
                for q in range(K):
                    b = int(np.sum(M[:q]))
                    e = int(np.sum(M[:q + 1]))
                    phi[b:e] -= (sro[q] - sro[k]) * 1e-6 * Ns
        self._cPhase = ph

    def _flags_for(self, s, f, k, start):
        """Control bytes of one (scene, family, node) for a start round
        (-1: not started within the run); records startRound / nSolves."""
        p, R = self.p, self.R
        g = self._gateState[(s, f, k)]
        started = np.zeros(R, dtype=bool)
        if start >= 0:
            started[start:] = True
        self.startRound[s, f, k] = start
        solve = started & g['doSolve']
        # not yet started: perform_update leaves the init slot
        # wTilde[:, i + 1] in place (d_classes.py:2290-2362); it
        # differs from w[i] only for random init (flag INITSLOT)
        initslot = (~started) & g['doSolve'] & (p.filterInitType == 'random')
        if p.bypassUpdates:
            solve[:] = False
            initslot[:] = False
        self.nSolves[s, f, k] = int(solve.sum())
        b = g['opY'].astype(np.uint8) | (g['opN'].astype(np.uint8) << 2) | (solve.astype(np.uint8) * L.FLAG_SOLVE)
        b = b | (initslot.astype(np.uint8) * L.FLAG_INITSLOT)
        if g['extT'] is not None:
            b = b | (g['extT'].astype(np.uint8) * L.FLAG_EXT_TARGET)
        if self.pregiven is not None:
            b = np.full(R, L.FLAG_PREGIVEN, dtype=np.uint8)
        return b

    def _build_flags(self):
        p, S, K, R = self.p, self.S, self.K, self.R
        fl = np.zeros((R, S, 4, K), dtype=np.uint8)
        self._gateState = {}
        self.startRound = np.full((S, 4, K), -1, dtype=np.int64)
        self.nSolves = np.zeros((S, 4, K), dtype=np.int64)
        vad = np.zeros((S, K, R), dtype=bool)
        for s, sc in enumerate(self.scenes):
            for k, nd in enumerate(sc.wasn):
                v = nd.vadPerFrame
                if len(v) < R:
                    raise ValueError('vadPerFrame shorter than the number of rounds')
                vad[s, k] = v[:R]
        self.vad = vad
        cvad = (vad.astype(np.float64).sum(axis=1) / K).astype(bool)   # [S][R] (d_classes.py:905-911)
        nY = np.cumsum(vad, axis=2)          # counters after the increment of round r
        nN = np.arange(1, R + 1)[None, None, :] - nY
        doSolve = self.rt.doSolve.T.astype(bool)    # [K][R]
        t = self.rt.t                                # [R][K]
        tOK = t >= p.startUpdatesAfterAtLeast
        # external-filter target timer (asy)
        extT = np.zeros((R, K), dtype=bool)
        last = np.zeros(K)
        for r in range(R):
            for k in range(K):
                if t[r, k] - last[k] >= p.timeBtwExternalFiltUpdates:
                    extT[r, k] = True
                    last[k] = t[r, k]
        basis = p.use1stFrameAsBasis
        for f in self.fams:
            for k in range(K):
                D = self.Dfam[f][k]
                for s in range(S):
                    v = cvad[s] if f == L.FAM_CENTR else vad[s, k]
                    ny, nn = nY[s, k], nN[s, k]
                    if basis:
                        opY = np.where(v & (ny == 1), L.OP_SET, np.where(ny > 1, np.where(v, L.OP_AVG, L.OP_KEEP), L.OP_KEEP))
                        opN = np.where(~v & (nn == 1), L.OP_SET, np.where(nn > 1, np.where(~v, L.OP_AVG, L.OP_KEEP), L.OP_KEEP))
                    else:
                        opY = np.where(v, L.OP_AVG, L.OP_KEEP)
                        opN = np.where(~v, L.OP_AVG, L.OP_KEEP)
                    elig = (ny > D) & (nn > D) & tOK[:, k]
                    self._gateState[(s, f, k)] = dict(elig=elig, opY=opY, opN=opN, doSolve=doSolve[k],
                                                      extT=extT[:, k] if f == L.FAM_DANSE else None)
                    # compiled assuming the reference gate passes at the first
                    # round the counters allow (run() checks it on the device)
                    fl[:, s, f, k] = self._flags_for(s, f, k, int(np.argmax(elig)) if elig.any() else -1)
        self.flags = fl

    def _winit(self, f, k):
        """Initial filter history (F, nIter + 1, D) of family f ('ext': the
        external filters) at node k."""
        p = self.p
        if f == 'ext':
            D, ref = self.M[k], p.referenceSensor
        else:
            D, ref = self.Dfam[f][k], self.refFam[f][k]
        return init_filter_history(self.F, self.nIter, D, ref, p.filterInitType, p.filterInitFixedValue)

    def _build_cfg(self):
        p, S, K, F = self.p, self.S, self.K, self.F
        fi = dict(initType=p.filterInitType, fixedValue=p.filterInitFixedValue)
        w0 = []
        scm = []
        sls = init_scm_slices(p, self.Mtot, K, F)
        for f in [0, 1, 2, 3]:
            if f not in self.fams:
                continue
            for k in range(K):
                D = self.Dfam[f][k]
                w0.append(np.ascontiguousarray(self._winit(f, k)[:, 0, :]).ravel())
                scm.append(np.ascontiguousarray(sls[k][..., :D, :D]).ravel())
        self._w0 = _cf32(np.concatenate(w0))
        self._scm = np.ascontiguousarray(np.concatenate(scm).astype(np.complex128)).view(np.float64)
        ext = [np.ascontiguousarray(self._winit('ext', k)[:, 0, :]).ravel() for k in range(K)]
        self._wExt0 = _cf32(np.concatenate(ext))
        # wTildeExtTarget: its own (F, M) draw (d_classes.py:687-691)
        tgt = [init_complex_filter((F, self.M[k]), p.referenceSensor, **fi).ravel() for k in range(K)]
        self._tgt0 = _cf32(np.concatenate(tgt))
        extMode = []
        for k in range(K):
            if p.onlyBroadcastRefSensorSigs:
                extMode.append(L.EXT_REFONLY)
            elif self.M[k] == 1 and p.noFusionAtSingleSensorNodes:
                extMode.append(L.EXT_KEEP)
            elif p.noExternalFilterRelaxation or 'seq' in p.nodeUpdating:
                extMode.append(L.EXT_COPY)
            else:
                extMode.append(L.EXT_RELAX)
        self._extMode = np.array(extMode, dtype=np.int32)
        beta = np.zeros((S, K), dtype=np.float64)
        betaE = np.zeros((S, K), dtype=np.float32)
        for s, sc in enumerate(self.scenes):
            for k, nd in enumerate(sc.wasn):
                beta[s, k] = p.forcedBeta if p.forcedBeta is not None else beta_from_t50p(p.t_expAvg50p, nd.fs, self.Ns)
                betaE[s, k] = (p.forcedBetaExternalFilters if p.forcedBetaExternalFilters is not None
                               else beta_from_t50p(p.t_expAvg50pExternalFilters, nd.fs, self.Ns))
        self._beta, self._betaE = beta, betaE
        self._M = np.array(self.M, dtype=np.int32)
        self._hA = np.asarray(p.winWOLAanalysis, dtype=np.float32)
        self._hS = np.asarray(p.winWOLAsynthesis, dtype=np.float32)
        self._bc = np.ascontiguousarray(self.rt.bcEnd.astype(np.int32))
        self._up = np.ascontiguousarray(self.rt.upEnd.astype(np.int32))
        self._flags = np.ascontiguousarray(self.flags)
        c = L.DanseCfg()
        c.S, c.K, c.M = S, K, _ptr(self._M, ctypes.c_int32)
        c.N, c.Ns, c.T, c.R = self.N, self.Ns, self.T, self.R
        c.k0, c.k1 = self.k0, self.k1
        c.gevd, c.rank, c.ref = int(bool(p.performGEVD)), int(p.GEVDrank), int(p.referenceSensor)
        c.families = self.famMask
        c.alphaExt = float(p.alphaExternalFilters)
        c.extMode = _ptr(self._extMode, ctypes.c_int32)
        c.beta, c.betaExt = _ptr(self._beta, ctypes.c_double), _ptr(self._betaE, ctypes.c_float)
        c.winAnalysis, c.winSynthesis = _ptr(self._hA, ctypes.c_float), _ptr(self._hS, ctypes.c_float)
        c.bcEnd, c.upEnd = _ptr(self._bc, ctypes.c_int32), _ptr(self._up, ctypes.c_int32)
        c.flags = _ptr(self._flags, ctypes.c_uint8)
        c.w0, c.wExt0, c.wExtTarget0 = (_ptr(self._w0, ctypes.c_float), _ptr(self._wExt0, ctypes.c_float),
                                        _ptr(self._tgt0, ctypes.c_float))
        c.scmInit = _ptr(self._scm, ctypes.c_double)
        c.keepHistory = int(bool(self.keepHistory))
        c.smallDGrid = int(self.smallDGrid)
        c.zLag = _ptr(self._zLag, ctypes.c_uint8)
        c.zPhase = _ptr(self._zPhase, ctypes.c_double)
        self._fsTab = np.ascontiguousarray(self.rt.fsTab, dtype=np.int32) if self.fewSamples else None
        c.fsTab = _ptr(self._fsTab, ctypes.c_int32)
        if self.fewSamples:
            # the step list (chunk appends, analyses, node-subset updates in
            # the reference's dependency order) and its chunk rows, padded to
            # the fsTab field layout
            ev = self.rt.fsEv
            rows = np.zeros((max(len(ev), 1), K, FS_FIELDS), dtype=np.int32)
            rows[:, :, FS_IRSRC] = -1
            rows[:len(ev), :, :4] = ev
            self._fsEv = np.ascontiguousarray(rows)
            self._fsSteps = np.ascontiguousarray(self.rt.fsSteps, dtype=np.int32)
            c.fsEv, c.nFsEv = _ptr(self._fsEv, ctypes.c_int32), int(len(ev))
            c.fsSteps, c.nFsSteps = _ptr(self._fsSteps, ctypes.c_int32), int(len(self._fsSteps))
        c.scmInitPerBin = 0 if p.covMatSameInitForAllFreqs else 1
        if self.cohDrift:
            cd = p.cohDrift
            c.cohDrift, c.cdSegLength, c.cdEvery = (2 if cd.loop == 'open' else 1), int(cd.segLength), int(cd.estEvery)
            if self._cdFlagWin is not None:
                c.cdFlagWin = _ptr(self._cdFlagWin, ctypes.c_double)
            c.cdStart = int(cd.startAfterNups + cd.estEvery)
            c.cdCompensate = int(bool(p.compensateSROs))
            c.cdNIter = int(self.nIter)
            c.cdAlpha, c.cdAlphaEps = float(cd.alpha), float(cd.alphaEps)
        if self.dxcp:
            c.dxcp = 1
            c.cdCompensate = int(bool(p.compensateSROs))
        c.cEnd = _ptr(self._cEnd, ctypes.c_int32)
        c.rawStreams = int(self._rawStreams)
        # 'conv': T(z) time-domain estimates (get_desired_sig_chunk, d_base.py:2085-2100)
        c.desSigConv = int(p.desSigProcessingType == 'conv')
        c.cPhase = _ptr(self._cPhase, ctypes.c_double)
        c.zStreamLen = int(self.rt.zStreamLen) if self.fewSamples else 0
        self.zLen = c.zStreamLen if self.fewSamples else self.R * self.Ns
        self._cfg = c
        eng = ctypes.c_void_p()
        L.check(self.lib.danse_engine_create(ctypes.byref(c), int(self.device), ctypes.byref(eng)))
        self.eng = eng

    def _load_pregiven(self, pg):
        """Load recorded filter histories (reference layout [F][nIter+1][D])."""
        R, F = self.R, self.F
        name = {L.FAM_DANSE: 'internalFilters', L.FAM_LOCAL: 'filtersLocal', L.FAM_CENTR: 'filtersCentr',
                L.FAM_SSBC: 'filtersSSBC'}
        for f in self.fams:
            for k in range(self.k0, self.k1):
                D = self.Dfam[f][k]
                arr = np.empty((self.S, R + 1, F, D), dtype=np.complex64)
                for s in range(self.S):
                    src = pg[s][name[f]][k] if isinstance(pg, (list, tuple)) else getattr(pg, name[f])[k]
                    arr[s] = np.transpose(src[:, :R + 1, :], (1, 0, 2))
                self._put(L.OUT_W, f, k, arr)
        for k in range(self.k0, self.k1):
            M = self.M[k]
            arr = np.empty((self.S, R + 1, F, M), dtype=np.complex64)
            for s in range(self.S):
                src = pg[s]['externalFilters'][k] if isinstance(pg, (list, tuple)) else pg.externalFilters[k]
                arr[s] = np.transpose(src[:, :R + 1, :], (1, 0, 2))
            self._put(L.OUT_WEXT, 0, k, arr)

    def _put(self, which, fam, node, arr):
        arr = np.ascontiguousarray(arr)
        L.check(self.lib.danse_engine_put(self.eng, which, fam, node, arr.ctypes.data_as(ctypes.c_void_p),
                                          arr.nbytes, None), self.eng)

    # ------------------------------------------------------------------ #
    def stream_ptr(self, stream=None):
        t = self.torch
        st = stream if stream is not None else t.cuda.current_stream(self.device)
        return ctypes.c_void_p(st.cuda_stream)

    def run(self, graph=True, stream=None, gate=True, reset=True):
        """The whole run, from the initial state (``reset``: the state reset
        of danse_engine_reset first; a fresh engine starts there anyway).
        ``gate``: the reference's start gate (Hermitian /
        positive definite / full rank over every bin, ``check_covariance_
        matrices``, ``d_classes.py:1430-1540``) is evaluated on the device at
        each family-node's first counter-eligible round.  Speculatively first:
        the checks run inside the (graph-captured) run, whose solve flags
        assume every check passes, and the verdicts are read back once; if
        one failed, the run is repeated exactly with the host loop
        (``_run_gated``: un-graphed up to the last decision, the start and
        the solve flags moved to the first round that passes)."""
        st = self.stream_ptr(stream)
        if self._ran:
            self._load_init_history()   # the solves of the previous run overwrote init slots
            self._reset_gate()
            if reset:
                L.check(self.lib.danse_engine_reset(self.eng, st), self.eng)
        self._ran = True
        gating = gate and self.pregiven is None and not self.p.bypassUpdates
        if gating and not self._gateSpecFailed:
            n = self._install_gate()
            if self.resident:
                self._run_resident(st)
            else:
                L.check(self.lib.danse_engine_run(self.eng, 0, self.R, st, int(bool(graph))), self.eng)
            if n == 0:
                return self
            ver = np.zeros(n, dtype=np.int32)
            L.check(self.lib.danse_engine_gate_verdicts(self.eng, _ptr(ver, ctypes.c_int32), st), self.eng)
            if np.all(ver != 0):
                return self
            # a start is delayed: repeat the run exactly on the host loop
            self._gateSpecFailed = True
            L.check(self.lib.danse_engine_reset(self.eng, st), self.eng)
            self._load_init_history()
        if gating:
            self._uninstall_gate()
            r0 = self._run_gated(st)
        else:
            if self.resident:
                self._run_resident(st)
                return self
            r0 = 0
        if r0 < self.R:
            L.check(self.lib.danse_engine_run(self.eng, r0, self.R, st, int(bool(graph))), self.eng)
        else:
            L.check(self.lib.danse_engine_finish(self.eng, st), self.eng)
        return self

    def _run_resident(self, st):
        """One persistent launch for the whole run (resident engine); raises
        if a wave gave up waiting (a hand-off that never arrived)."""
        L.check(self.lib.danse_engine_run_resident(self.eng, st), self.eng)
        err = ctypes.c_int32()
        L.check(self.lib.danse_engine_resident_error(self.eng, ctypes.byref(err), st), self.eng)
        if err.value:
            raise RuntimeError('resident run: a wave gave up waiting for a hand-off')

    def _gate_candidates(self):
        """(round, (s, f, k)) of every owned family-node's first counter-eligible round."""
        out = []
        for key, g in self._gateState.items():
            if key[2] < self.k0 or key[2] >= self.k1:
                continue
            e = np.flatnonzero(g['elig'])
            if e.size:
                out.append((int(e[0]), key))
        return out

    def _install_gate(self):
        if self._gateInstalled is not None:
            return self._gateInstalled
        cands = self._gate_candidates()
        n = len(cands)
        rnd = np.array([c[0] for c in cands], dtype=np.int32)
        scn = np.array([c[1][0] for c in cands], dtype=np.int32)
        fam = np.array([c[1][1] for c in cands], dtype=np.int32)
        node = np.array([c[1][2] for c in cands], dtype=np.int32)
        qY = np.array([self._gate_q(s, k, self._gateState[(s, f, k)]['opY'], r) for r, (s, f, k) in cands])
        qN = np.array([self._gate_q(s, k, self._gateState[(s, f, k)]['opN'], r) for r, (s, f, k) in cands])
        L.check(self.lib.danse_engine_set_gate(self.eng, n, _ptr(rnd, ctypes.c_int32), _ptr(fam, ctypes.c_int32),
                                               _ptr(node, ctypes.c_int32), _ptr(scn, ctypes.c_int32),
                                               _ptr(qY, ctypes.c_double), _ptr(qN, ctypes.c_double)), self.eng)
        self.graph_gen += 1
        self._gateInstalled = n
        return n

    def _uninstall_gate(self):
        if self._gateInstalled:
            z = np.zeros(1, dtype=np.int32)
            d = np.zeros(1)
            L.check(self.lib.danse_engine_set_gate(self.eng, 0, _ptr(z, ctypes.c_int32), _ptr(z, ctypes.c_int32),
                                                   _ptr(z, ctypes.c_int32), _ptr(z, ctypes.c_int32),
                                                   _ptr(d, ctypes.c_double), _ptr(d, ctypes.c_double)), self.eng)
            self.graph_gen += 1
        self._gateInstalled = None

    def _reset_gate(self):
        if not self._gateMoved:
            return
        self._gateMoved = False
        fl = self.flags
        for (s, f, k), g in self._gateState.items():
            fl[:, s, f, k] = self._flags_for(s, f, k, int(np.argmax(g['elig'])) if g['elig'].any() else -1)
        self._flags = np.ascontiguousarray(fl)
        L.check(self.lib.danse_engine_set_flags(self.eng, _ptr(self._flags, ctypes.c_uint8), None), self.eng)
        self.graph_gen += 1

    def _gate_q(self, s, k, ops, r):
        """beta^m of the init slice's anti-Hermitian residue after round r
        (0 once a first-frame SET replaced the init)."""
        o = ops[:r + 1]
        if np.any(o == L.OP_SET):
            return 0.0
        return float(self._beta[s, k]) ** int(np.sum(o == L.OP_AVG))

    def _gate_pending(self):
        """{(s, f, k): first counter-eligible round} of every owned family-node."""
        pending = {}
        for key, g in self._gateState.items():
            if key[2] < self.k0 or key[2] >= self.k1:
                continue
            e = np.flatnonzero(g['elig'])
            if e.size:
                pending[key] = int(e[0])
        return pending

    def _gate_decide(self, rc, pending, st, nodes=None):
        """The exact gate of round rc (after its broadcast, before its update):
        check every candidate pending at rc (of ``nodes``, default all) on the
        device, move the start (and the solve flags) of those that fail to
        their next eligible round, and upload the flags if they changed."""
        cands = sorted(key for key, r in pending.items() if r == rc and (nodes is None or key[2] in nodes))
        if not cands:
            return
        fam = np.array([c[1] for c in cands], dtype=np.int32)
        node = np.array([c[2] for c in cands], dtype=np.int32)
        scn = np.array([c[0] for c in cands], dtype=np.int32)
        qY = np.array([self._gate_q(c[0], c[2], self._gateState[c]['opY'], rc) for c in cands])
        qN = np.array([self._gate_q(c[0], c[2], self._gateState[c]['opN'], rc) for c in cands])
        ver = np.zeros(len(cands), dtype=np.int32)
        L.check(self.lib.danse_engine_gate(self.eng, rc, len(cands), _ptr(fam, ctypes.c_int32),
                                           _ptr(node, ctypes.c_int32), _ptr(scn, ctypes.c_int32),
                                           _ptr(qY, ctypes.c_double), _ptr(qN, ctypes.c_double),
                                           _ptr(ver, ctypes.c_int32), st), self.eng)
        changed = False
        for c, v in zip(cands, ver):
            s, f, k = c
            if v:
                del pending[c]
                if self.startRound[s, f, k] != rc:
                    self.flags[:, s, f, k] = self._flags_for(s, f, k, rc)
                    changed = True
            else:
                nxt = np.flatnonzero(self._gateState[c]['elig'][rc + 1:])
                if nxt.size:
                    pending[c] = rc + 1 + int(nxt[0])
                else:
                    del pending[c]
                if self.startRound[s, f, k] != -1:
                    self.flags[:, s, f, k] = self._flags_for(s, f, k, -1)
                    changed = True
        if changed:
            self._gateMoved = True
            self._flags = np.ascontiguousarray(self.flags)
            L.check(self.lib.danse_engine_set_flags(self.eng, _ptr(self._flags, ctypes.c_uint8), st), self.eng)
            self.graph_gen += 1

    def _split_round(self, r):
        """fewSamples: round r's updates run as several node-subset steps."""
        if not self.fewSamples:
            return False
        rs = self.rt.fsRoundStep
        return int(np.count_nonzero(self.rt.fsSteps[rs[r]:rs[r + 1], 0] == FS_STEP_UPDATE)) > 1

    def _run_gated(self, st):
        R = self.R
        pending = self._gate_pending()
        r0 = 0
        while pending:
            rc = min(pending.values())
            if rc > r0:
                L.check(self.lib.danse_engine_run(self.eng, r0, rc, st, 0), self.eng)
            if self._split_round(rc):
                # each node's gate right before its own update step (its z
                # frames may be analysed only after another node's update)
                rs = self.rt.fsRoundStep
                i0 = int(rs[rc])
                for i in range(int(rs[rc]), int(rs[rc + 1])):
                    ty, _, mask, _ = (int(x) for x in self.rt.fsSteps[i])
                    if ty == FS_STEP_UPDATE:
                        L.check(self.lib.danse_engine_run_steps(self.eng, i0, i, st), self.eng)
                        self._gate_decide(rc, pending, st, nodes={k for k in range(self.K) if (mask >> k) & 1})
                        i0 = i
                L.check(self.lib.danse_engine_run_steps(self.eng, i0, int(rs[rc + 1]), st), self.eng)
            else:
                L.check(self.lib.danse_engine_bcast(self.eng, rc, st), self.eng)
                self._gate_decide(rc, pending, st)
                L.check(self.lib.danse_engine_update(self.eng, rc, st), self.eng)
            r0 = rc + 1
            if r0 >= R:
                break
        return r0

    # ---- the gate for callers that sequence the rounds themselves (the
    # node-sharded runner, danse_amd.dist.ShardedRun)
    def gating(self, gate=True):
        return bool(gate and self.pregiven is None and not self.p.bypassUpdates)

    def begin_run(self, speculative, stream=None):
        """State bookkeeping before a caller-sequenced run: re-load the init
        slots a previous run's solves overwrote, restore the counter-compiled
        flags, and install (speculative) or remove (exact) the in-run gate."""
        if self._ran:
            self._load_init_history()
            self._reset_gate()
        self._ran = True
        if speculative:
            return self._install_gate()
        self._uninstall_gate()
        return 0

    def gate_launch(self, r, stream=None):
        """Speculative gate of round r (between the all-gather and update(r))."""
        L.check(self.lib.danse_engine_gate_launch(self.eng, int(r), self.stream_ptr(stream)), self.eng)

    def gate_ok(self, stream=None):
        """True if every speculative gate check of the run passed."""
        n = self._gateInstalled or 0
        if n == 0:
            return True
        ver = np.zeros(n, dtype=np.int32)
        L.check(self.lib.danse_engine_gate_verdicts(self.eng, _ptr(ver, ctypes.c_int32), self.stream_ptr(stream)),
                self.eng)
        return bool(np.all(ver != 0))

    def mark_gate_failed(self):
        """A speculative run (on this or another rank) had a failing check:
        from now on the engine runs the exact host-gated sequence."""
        self._gateSpecFailed = True

    @property
    def gate_spec_failed(self):
        return self._gateSpecFailed

    def gate_pending(self):
        return self._gate_pending()

    def gate_decide(self, r, pending, stream=None, nodes=None):
        self._gate_decide(r, pending, self.stream_ptr(stream), nodes=nodes)

    def bcast(self, r, stream=None):
        L.check(self.lib.danse_engine_bcast(self.eng, r, self.stream_ptr(stream)), self.eng)

    def update(self, r, seg=None, stream=None):
        """The update phase of round r, or its segment ``seg`` (see
        ``update_segments``)."""
        if seg is None:
            L.check(self.lib.danse_engine_update(self.eng, r, self.stream_ptr(stream)), self.eng)
            return
        s0, s1, _ = self._segments(r)[seg]
        L.check(self.lib.danse_engine_run_steps(self.eng, s0, s1, self.stream_ptr(stream)), self.eng)

    def _segments(self, r):
        """fewSamples: the update phase of round r cut before each UPDATE
        step, [(first step, end step, node set)]."""
        rs = self.rt.fsRoundStep
        ups = [i for i in range(int(rs[r]), int(rs[r + 1])) if int(self.rt.fsSteps[i, 0]) == FS_STEP_UPDATE]
        ends = ups[1:] + [int(rs[r + 1])]
        return [(u, e, {k for k in range(self.K) if (int(self.rt.fsSteps[u, 2]) >> k) & 1})
                for u, e in zip(ups, ends)]

    def update_segments(self, r):
        """Number of update segments of round r: 1, or (a fewSamples round
        whose updates run as several node-subset steps) one per UPDATE step,
        each needing the z frames analysed after the previous one -- a
        node-sharded run exchanges the fused spectra before each segment."""
        return len(self._segments(r)) if self._split_round(r) else 1

    def segment_nodes(self, r, seg):
        """The nodes updated by segment ``seg`` of round r."""
        if not self._split_round(r):
            return set(range(self.K))
        return self._segments(r)[seg][2]

    def finish(self, stream=None):
        L.check(self.lib.danse_engine_finish(self.eng, self.stream_ptr(stream)), self.eng)

    def zspec(self):
        ptr = ctypes.c_void_p()
        nb = ctypes.c_size_t()
        L.check(self.lib.danse_engine_zspec(self.eng, ctypes.byref(ptr), ctypes.byref(nb)), self.eng)
        return ptr.value, nb.value

    def _get(self, which, fam=0, node=0, dtype=np.complex64, shape=None):
        nb = ctypes.c_size_t()
        L.check(self.lib.danse_engine_output_bytes(self.eng, which, fam, node, ctypes.byref(nb)), self.eng)
        out = np.empty(nb.value // np.dtype(dtype).itemsize, dtype=dtype)
        L.check(self.lib.danse_engine_get(self.eng, which, fam, node, out.ctypes.data_as(ctypes.c_void_p),
                                          out.nbytes, None), self.eng)
        return out.reshape(shape) if shape is not None else out

    def diagnostics(self):
        return self._get(L.OUT_DIAG, dtype=np.int32, shape=(self.S, self.K, 4))

    def lanczos_stats(self):
        """[R][2] int32 of the last run: per round, the bins whose warm-started
        rank-1 Lanczos solve was accepted and the bins its acceptance test sent
        back to the Householder path (lane-grid GEVD classes of DMAX >= 20;
        zeros elsewhere)."""
        out = np.zeros((self.R, 2), dtype=np.int32)
        L.check(self.lib.danse_engine_lanczos_stats(
            self.eng, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), out.size), self.eng)
        return out

    def dxcp_record(self, on=True):
        """Record every DXCP-PhaT feed's gathered input frames and estimator
        outputs over the following runs (estimateSROs='DXCPPhaT')."""
        L.check(self.lib.danse_engine_dxcp_record(self.eng, int(bool(on))), self.eng)

    def dxcp_recorded(self):
        """(frames [feeds][S][nOwn][K-1][2][2048] float32 -- channel 0 the
        receiver's reference sensor, 1 the sender's received z stream --,
        outputs [feeds][S][nOwn][K-1][2] float64 -- SRO ppm, STO samples) of
        the last recorded run; sender q of slot qi is qi + (qi >= k)."""
        nf, npair = ctypes.c_int32(), ctypes.c_int32()
        L.check(self.lib.danse_engine_dxcp_recorded(self.eng, ctypes.byref(nf), ctypes.byref(npair), None, 0, None,
                                                    0), self.eng)
        fr = np.empty((nf.value, npair.value, 2, 2048), dtype=np.float32)
        out = np.empty((nf.value, npair.value, 2), dtype=np.float64)
        if nf.value:
            L.check(self.lib.danse_engine_dxcp_recorded(self.eng, ctypes.byref(nf), ctypes.byref(npair),
                                                        fr.ctypes.data_as(ctypes.c_void_p), fr.nbytes,
                                                        out.ctypes.data_as(ctypes.c_void_p), out.nbytes), self.eng)
        shp = (nf.value, self.S, self.k1 - self.k0, self.K - 1)
        return fr.reshape(shp + (2, 2048)), out.reshape(shp + (2,))

    # ------------------------------------------------------------------ #
    def outputs(self):
        """Per scene, the ``dv`` fields in the reference layout."""
        p, S, K, F, R = self.p, self.S, self.K, self.F, self.R
        nI = self.nIter
        fi = dict(initType=p.filterInitType, fixedValue=p.filterInitFixedValue)
        res = [DanseOutputs() for _ in range(S)]
        hist = R + 1 if self.keepHistory else 2
        fname = {L.FAM_DANSE: ('wTilde', 'd', 'dhat'), L.FAM_LOCAL: ('wLocal', 'dLocal', 'dHatLocal'),
                 L.FAM_CENTR: ('wCentr', 'dCentr', 'dHatCentr'), L.FAM_SSBC: ('wSSBC', 'dSSBC', 'dHatSSBC')}
        for f in self.fams:
            wn, dn, dhn = fname[f]
            d = self._get(L.OUT_D, f, dtype=np.float32, shape=(S, K, self.T))
            dh = self._get(L.OUT_DHAT, f, shape=(S, K, R, F))
            for s in range(S):
                setattr(res[s], dn, d[s].T.astype(np.float64))
                full = np.zeros((F, nI, K), dtype=np.complex128)
                full[:, :R, :] = np.transpose(dh[s], (2, 1, 0))
                setattr(res[s], dhn, full)
                setattr(res[s], wn, [None] * K)
            for k in range(self.k0, self.k1):
                D = self.Dfam[f][k]
                w = self._get(L.OUT_W, f, k, shape=(S, hist, F, D))
                init = self._winit(f, k)
                for s in range(S):
                    full = np.empty((F, nI + 1, D), dtype=np.complex128)
                    full[:] = init
                    if self.keepHistory:
                        full[:, :R + 1, :] = np.transpose(w[s], (1, 0, 2))
                    getattr(res[s], wn)[k] = full
        z = self._get(L.OUT_Z, dtype=np.float32, shape=(S, K, self.zLen))
        for s in range(S):
            # fewSamples: the broadcast streams (the reference leaves zFullTD empty)
            res[s].zFullTD = [z[s, k].astype(np.float64) for k in range(K)]
            res[s].wTildeExt = [None] * K
        for k in range(self.k0, self.k1):
            M = self.M[k]
            e = self._get(L.OUT_WEXT, 0, k, shape=(S, hist, F, M))
            init = self._winit('ext', k)
            for s in range(S):
                full = np.empty((F, nI + 1, M), dtype=np.complex128)
                full[:] = init
                if self.keepHistory:
                    full[:, :R + 1, :] = np.transpose(e[s], (1, 0, 2))
                res[s].wTildeExt[k] = full
        diag = self.diagnostics()
        cond = self._cond_numbers() if self.condEvery else None
        # yinSTFT / yCentrBatch (d_classes.py:915-930): the whole-signal STFT of
        # the engine's inputs on the device, [S][F][nseg][Mtot]
        nseg = stft_frames(self.T, self.N, self.Ns)
        win = self.torch.from_numpy(np.asarray(p.winWOLAanalysis, dtype=np.float32)).to(self.y.device)
        Y = self.torch.empty((S, F, nseg, self.Mtot, 2), dtype=self.torch.float32, device=self.y.device)
        L.check_batch(self.lib.danse_stft(ctypes.c_void_p(self.y.data_ptr()), S, self.Mtot, self.T, self.N, self.Ns, nseg,
                                    ctypes.c_void_p(win.data_ptr()), ctypes.c_void_p(Y.data_ptr()),
                                    self.stream_ptr()))
        self.torch.cuda.synchronize(self.y.device)
        Yh = Y.cpu().numpy()
        Yh = Yh[..., 0].astype(np.float64) + 1j * Yh[..., 1].astype(np.float64)
        solveFlags = (self.flags[:, :, L.FAM_DANSE, :] & L.FLAG_SOLVE) != 0     # [R][S][K]
        neighbors0 = [list(n.neighborsIdx) for n in self.scenes[0].wasn]
        if self.cohDrift or self.dxcp:
            cdE = np.zeros((S, K, self.R, K - 1))
            cdR = np.zeros((S, K, self.R, K - 1))
            L.check(self.lib.danse_engine_sro_estimates(self.eng, _ptr(cdE, ctypes.c_double),
                                                        _ptr(cdR, ctypes.c_double)), self.eng)
        for s in range(S):
            r = res[s]
            kr = p.referenceSensor
            fsr = -1
            if kr < K and solveFlags[:, s, kr].any():
                fsr = int(np.argmax(solveFlags[:, s, kr]))
            for nm, v in host_fields(p, [n.sro for n in self.scenes[s].wasn], neighbors0, self.rt, nI, nseg,
                                     fsr).items():
                setattr(r, nm, v)
            if self.cohDrift or self.dxcp:
                r.SROsEstimates = [np.zeros((nI, K - 1)) for _ in range(K)]
                r.SROsResiduals = [np.zeros((nI, K - 1)) for _ in range(K)]
                for k in range(K):
                    r.SROsEstimates[k][:self.R] = cdE[s, k]
                    r.SROsResiduals[k][:self.R] = cdR[s, k]
            r.yCentrBatch = Yh[s]
            r.yinSTFT = [Yh[s][:, :, self.base[k]:self.base[k] + self.M[k]] for k in range(K)]
            r.computeCentralised = bool(p.computeCentralised)
            r.computeLocal = bool(p.computeLocal)
            r.computeSingleSensorBroadcast = bool(p.computeSingleSensorBroadcast)
            r.condNumbers = cond[s] if cond is not None else None
            r.startUpdates = self.startRound[s, 0] >= 0
            r.startRound = self.startRound[s, 0].copy()
            r.nInternalFilterUps = self.nSolves[s, 0].astype(np.float64)
            r.diag = diag[s]
            r.oVADframes = [self.scenes[s].wasn[k].vadPerFrame for k in range(K)]
            r.neighbors = [list(n.neighborsIdx) for n in self.scenes[s].wasn]
            r.fs = np.array([n.fs for n in self.scenes[s].wasn])
            r.SROsppm = np.array([n.sro for n in self.scenes[s].wasn])
            r.yin = [n.data for n in self.scenes[s].wasn]
            r.timeInstants = np.stack([n.timeStamps for n in self.scenes[s].wasn], axis=1)
            r.expAvgBeta = list(self._beta[s].astype(np.float64))
            r.cleanSpeechSignalsAtNodes = [n.cleanspeech for n in self.scenes[s].wasn]
            r.nIter = nI
            r.nRounds = R
        return res

    def _cond_numbers(self):
        """Per scene, the reference's ConditionNumbers fields
        (d_classes.py:19-130, 965-984): cn_Ryy{DANSE,Local,Centr}[k] (F,
        saves) and iter_cn_*[k] (the iterations), for the owned nodes."""
        import types
        S, K, F, R = self.S, self.K, self.F, self.R
        nOwn = self.k1 - self.k0
        nFN = len(self.fams) * nOwn
        h = np.empty(S * nFN * R * F)
        L.check(self.lib.danse_engine_cond(self.eng, h.ctypes.data_as(ctypes.c_void_p), h.nbytes), self.eng)
        h = h.reshape(S, nFN, R, F)
        it = [r for r in range(R) if (r + 1) % self.condEvery == 0]
        names = {L.FAM_DANSE: 'DANSE', L.FAM_LOCAL: 'Local', L.FAM_CENTR: 'Centr'}
        out = []
        for s in range(S):
            cn = types.SimpleNamespace()
            for nm in names.values():
                setattr(cn, f'cn_Ryy{nm}', [np.empty((F, 0)) for _ in range(K)])
                setattr(cn, f'iter_cn_Ryy{nm}', [[] for _ in range(K)])
            cn.cn_RyyDANSEcomputed = True
            cn.cn_RyyLocalComputed = bool(self.p.computeLocal)
            cn.cn_RyyCentrComputed = bool(self.p.computeCentralised)
            for fi, fam in enumerate(self.fams):
                if fam not in names:
                    continue
                for j, k in enumerate(range(self.k0, self.k1)):
                    getattr(cn, f'cn_Ryy{names[fam]}')[k] = h[s, fi * nOwn + j][it].T.copy()
                    getattr(cn, f'iter_cn_Ryy{names[fam]}')[k] = list(it)
            out.append(cn)
        return out

    def close(self):
        if getattr(self, 'eng', None):
            self.lib.danse_engine_destroy(self.eng)
            self.eng = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DanseOutputs:
    """Container with the reference's ``DANSEvariables`` output field names."""
    pass
