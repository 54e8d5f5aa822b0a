"""Host event scheduler — stays on the CPU.

Restates the reference's event-matrix construction for fully connected WASNs:
``initialize_events`` (``danse_toolbox/d_base.py:513-571``),
``base_event_checks``/``check_clock_jitter`` (``d_base.py:454-510``),
``prep_evmat_build`` fully connected branch (``d_base.py:797-889``),
``generate_aligned_instants`` (``d_base.py:892-920``),
``build_events_matrix`` (``d_base.py:962-1225``),
``sort_simultaneous_events`` (``d_base.py:1228-1334``) and
``events_groupping_check`` (``d_base.py:1337-1388``).

Everything is float64 and uses the reference's own operations so that event
instants, their grouping (exact float equality) and the integer frame ends
``floor(t * fs)`` are bit-identical (quirk Q3).  The GPU engine never sees a
float time: ``compile_rounds`` turns the event list into integer tables.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

EVENT_CODES = {'tr': -1, 'fu': 0, 'bc': 1, 're': 2, 'up': 3}
_REV = {v: k for k, v in EVENT_CODES.items()}


@dataclass
class DANSEeventInstant:
    """``d_base.py:40-52``."""
    t: float = 0.
    nodes: np.ndarray = field(default_factory=lambda: np.array([0]))
    type: list = field(default_factory=list)
    bypassUpdate: list = field(default_factory=list)

    def __post_init__(self):
        self.nEvents = len(self.nodes)


def check_clock_jitter(timeInstants: np.ndarray, nNodes: int) -> np.ndarray:
    fs = np.zeros(nNodes)
    for k in range(nNodes):
        deltas = np.diff(timeInstants[:, k])
        precision = int(np.ceil(np.abs(np.log10(np.mean(deltas) / 1e4))))
        u = np.unique(np.round(deltas, precision))
        if len(u) > 1:
            raise ValueError(f'[NOT IMPLEMENTED] Clock jitter detected: {len(u)} different sample intervals detected for node {k + 1}.')
        fs[k] = np.round(1 / u[0], 3)
    return fs


def generate_aligned_instants(startIdx, eventSep, nEventTotal, timeStamps, fsNodes):
    ev = [np.arange(startIdx, int(nEventTotal[k])) * eventSep / fsNodes[k] for k in range(len(timeStamps))]
    for k in range(len(timeStamps)):
        instants = timeStamps[k]
        inset = set(instants.tolist())
        for ii in range(len(ev[k])):
            if ev[k][ii] not in inset:
                possible = instants[instants > ev[k][ii]]
                ev[k][ii] = possible[0] if len(possible) > 0 else instants[-1]
    return ev


def initialize_events(timeStamps: list, nodeFs: list, p, neighbors: list):
    """Returns ``(events, fs)``; ``timeStamps[k]`` is node k's sample clock,
    ``nodeFs[k]`` its true (SRO-affected) rate (``Node.fs``)."""
    T = np.stack(timeStamps, axis=1)
    nNodes = T.shape[1]
    fs = check_clock_jitter(T, nNodes)
    if 'sim' in p.nodeUpdating and any(fs != fs[p.referenceSensor]):
        raise ValueError('Simultaneous node-updating impossible in the presence of SROs.')
    if 'topo-indep' in p.nodeUpdating:
        raise NotImplementedError('TI-DANSE (ad-hoc topologies) is out of scope (SURVEY §8f row 4).')
    Ttot = T[-1, :]
    numPotentialUpInTtot = np.floor(Ttot * fs / p.Ns)
    numBcInTtot = np.floor(Ttot * fs / p.broadcastLength)
    if p.broadcastType == 'wholeChunk':
        bc = generate_aligned_instants(p.DFTsize / p.broadcastLength, p.Ns, numBcInTtot, timeStamps, nodeFs)
        up = generate_aligned_instants(np.ceil(p.DFTsize / p.Ns), p.Ns, numPotentialUpInTtot, timeStamps, nodeFs)
    elif p.broadcastType == 'fewSamples':
        up = generate_aligned_instants(np.ceil(p.DFTsize / p.Ns), p.Ns, numPotentialUpInTtot, timeStamps, nodeFs)
        if p.efficientSpSBC:
            bc = []
            for k in range(nNodes):
                comb = []
                for q in neighbors[k]:
                    for x in up[q]:
                        if x not in comb:
                            comb.append(x)
                bc.append(np.sort(np.array(comb)))
            for k in range(nNodes):
                possibleBc = timeStamps[k][int(p.broadcastLength)::int(p.broadcastLength)]
                pset = set(possibleBc.tolist())
                for ii in range(len(bc[k])):
                    if bc[k][ii] not in pset:
                        pi = possibleBc[possibleBc < bc[k][ii]]
                        bc[k][ii] = pi[-1] if len(pi) > 0 else possibleBc[0]
        else:
            bc = generate_aligned_instants(1, p.broadcastLength, numBcInTtot, timeStamps, nodeFs)
    else:
        raise ValueError(f'Unknown broadcast type {p.broadcastType}')
    events = build_events_matrix(up, bc, p.nodeUpdating, p.seqUpdateStartNodeIdx, p.updateEvery)
    return events, fs


def _flatten(K, t, code):
    if len(t) == 0:
        return np.zeros((0, 3))
    n = int(np.sum([len(np.unique(t[k])) for k in range(K)]))
    out = np.zeros((n, 3))
    for k in range(K):
        s = int(np.sum([len(np.unique(t[q])) for q in range(k)]))
        u = np.unique(t[k])
        out[s:s + len(u), 0] = u
        out[s:s + len(u), 1] = k
        out[:, 2] = code
    return out


def build_events_matrix(up_t, bc_t, nodeUpdating='seq', firstUpdatingNode=0, minNumFramesBwUpdates=0):
    nNodes = len(up_t)
    upI = _flatten(nNodes, up_t, EVENT_CODES['up'])
    bcI = _flatten(nNodes, bc_t, EVENT_CODES['bc'])
    ev = np.concatenate((upI, bcI), axis=0)
    # np.argsort default (quicksort) as the reference: ties keep the concatenation
    # order only where quicksort does; we reproduce the exact call.
    ev = ev[np.argsort(ev[:, 0], axis=0), :]
    nEv = ev.shape[0]
    out = []
    idx = 0
    lastUpNode = firstUpdatingNode - 1
    nFramesSinceLastUpdate = 0
    while idx < nEv:
        t0 = ev[idx, 0]
        nodes = [int(ev[idx, 1])]
        types = [int(ev[idx, 2])]
        # events_groupping_check (d_base.py:1337-1388)
        if idx < nEv - 1:
            nxt = ev[idx + 1, 0]
            cur = t0
            if cur == nxt:
                while cur == nxt:
                    idx += 1
                    cur = ev[idx, 0]
                    nodes.append(int(ev[idx, 1]))
                    types.append(int(ev[idx, 2]))
                    if idx < nEv - 1:
                        nxt = ev[idx + 1, 0]
                    else:
                        idx += 1
                        break
                else:
                    idx += 1
            else:
                idx += 1
        else:
            idx += 1
        nodes = np.array(nodes, dtype=int)
        types = np.array(types, dtype=int)
        # sort_simultaneous_events, fully connected branch (d_base.py:1326-1332)
        order = np.empty(0, dtype=int)
        base = np.arange(len(types))
        for key in ['tr', 'fu', 'bc', 're', 'up']:
            sel = base[types == EVENT_CODES[key]]
            if len(sel) > 0:
                sel = sel[np.argsort(nodes[sel])]
            order = np.concatenate((order, sel))
        nodes = nodes[order]
        types = [_REV[c] for c in types[order]]
        bypass = [False for _ in types]
        if 'up' in types:
            nFramesSinceLastUpdate += 1
            lastUpNodeUpdated = lastUpNode
            for ii in range(len(types)):
                if types[ii] == 'up':
                    if nFramesSinceLastUpdate < minNumFramesBwUpdates:
                        bypass[ii] = True
                    elif 'seq' in nodeUpdating:
                        if nodes[ii] == np.mod(lastUpNode + 1, nNodes):
                            lastUpNodeUpdated = nodes[ii]
                        else:
                            bypass[ii] = True
            if not all(np.array(bypass)[np.array(types) == 'up']):
                nFramesSinceLastUpdate = 0
            lastUpNode = lastUpNodeUpdated
        out.append(DANSEeventInstant(t=t0, nodes=nodes, type=types, bypassUpdate=bypass))
    return out


# --------------------------------------------------------------------------- #
# Integer round tables for the device engine
# --------------------------------------------------------------------------- #

@dataclass
class RoundTables:
    """Per-round integer schedule of fully connected wholeChunk DANSE.  Device
    round r = DANSE iteration r of every node: phase A runs every node's
    broadcast r, phase B every node's update r.

    bcEnd[r, k]    sample index one past the broadcast frame's end (floor(t fs))
    upEnd[r, k]    same for the update frame, already shifted by -(N - Ns)
    doSolve[r, k]  1 if the filter update is not bypassed (seq round robin)
    zLag[r, k, q]  0: node k's update r consumes sender q's fused frame of
                   round r; 1: of round r-1 (SRO clocks, quirk Q13)
    flags[r, k, q] full-sample-drift buffer flags (process_incoming_signals_
                   buffers, d_classes.py:1745-1807)
    nRounds        number of rounds (= DANSE iterations per node)
    t[r, k]        instant (reference time axis) of node k's update r
    synchronous    every node shares every instant (no SROs)
    """
    bcEnd: np.ndarray
    upEnd: np.ndarray
    doSolve: np.ndarray
    nRounds: int
    t: np.ndarray = None
    zLag: np.ndarray = None
    flags: np.ndarray = None
    synchronous: bool = True
    fsTab: np.ndarray = None      # fewSamples: [R][K][FS_FIELDS] (compile_rounds_fs)
    zStreamLen: int = 0


def compile_rounds(events, fs, p, nNodes: int) -> RoundTables:
    """Turns the reference event list into integer round tables.

    Replays the events in the reference's order (``d_core.py:66-90``) with
    the buffer bookkeeping of ``fill_buffers`` / ``process_incoming_signals_
    buffers`` (``d_classes.py:1185-1224,1701-1807``): every broadcast adds Ns
    samples to each neighbour's buffer, every update empties it.  The fused
    frame a node consumes is the last N received samples of the sender's
    stream; the device keeps the sender spectra of the last two rounds, so a
    schedule is accepted when every update consumes the sender's round r or
    r-1 frame (SRO drift below Ns samples).  Raises NotImplementedError for
    anything else (fewSamples broadcasts, larger drifts)."""
    if p.broadcastType != 'wholeChunk':
        raise NotImplementedError('fewSamples broadcasts are not on the device round path')
    K, N, Ns = nNodes, p.DFTsize, p.Ns
    bc = [[] for _ in range(K)]
    up = [[] for _ in range(K)]
    solve = [[] for _ in range(K)]
    tUp = [[] for _ in range(K)]
    buf = np.zeros((K, K), dtype=np.int64)      # buf[k, q]: samples from q waiting at k
    recv = np.zeros((K, K), dtype=np.int64)     # total samples of q's stream received by k
    lag = [[] for _ in range(K)]
    flg = [[] for _ in range(K)]
    sync = True
    for ev in events:
        ks = list(ev.nodes)
        if ev.type != ['bc'] * K + ['up'] * K or ks != list(range(K)) * 2:
            sync = False
        for ii, (k, typ) in enumerate(zip(ks, ev.type)):
            k = int(k)
            if typ == 'bc':
                if len(bc[k]) != len(up[k]):
                    raise NotImplementedError('two broadcasts of a node without an update in between')
                bc[k].append(int(np.floor(ev.t * fs[k])))
                for q in range(K):
                    if q != k:
                        buf[q, k] += Ns
                        recv[q, k] += Ns
            else:
                r = len(up[k])
                if len(bc[k]) != r + 1:
                    raise NotImplementedError('update without its broadcast')
                up[k].append(int(np.floor(ev.t * fs[k])) - (N - Ns))
                solve[k].append(0 if ev.bypassUpdate[ii] else 1)
                tUp[k].append(ev.t)
                lr = np.zeros(K, dtype=np.int64)
                fr = np.zeros(K, dtype=np.int64)
                for q in range(K):
                    if q == k:
                        continue
                    Bq = buf[k, q]
                    if r == 0:
                        fr[q] = 0 if Bq == N else (-(N - Bq) if Bq < N else (Bq - N))
                    else:
                        fr[q] = 0 if Bq == Ns else (-(Ns - Bq) if Bq < Ns else (Bq - Ns))
                    d = (r + 1) * Ns - recv[k, q]
                    if d not in (0, Ns):
                        raise NotImplementedError(f'node {k} update {r} consumes sender {q} {d} samples behind '
                                                  '(drift beyond one chunk)')
                    lr[q] = d // Ns
                    buf[k, q] = 0
                lag[k].append(lr)
                flg[k].append(fr)
    R = min(len(u) for u in up)
    if R < 1:
        return RoundTables(np.zeros((0, K), np.int64), np.zeros((0, K), np.int64), np.zeros((0, K), np.int32), 0,
                           np.zeros((0, K)), np.zeros((0, K, K), np.uint8), np.zeros((0, K, K), np.int64), sync)
    bcEnd = np.array([b[:R] for b in bc], dtype=np.int64).T
    upEnd = np.array([u[:R] for u in up], dtype=np.int64).T
    doSolve = np.array([x[:R] for x in solve], dtype=np.int32).T
    zLag = np.stack([np.stack(l[:R]) for l in lag], axis=1).astype(np.uint8)     # [R][K][K]
    flags = np.stack([np.stack(f[:R]) for f in flg], axis=1)                   # [R][K][K]
    t = np.array([x[:R] for x in tUp], dtype=np.float64).T
    return RoundTables(bcEnd, upEnd, doSolve, R, t, zLag, flags, sync)


FS_FIELDS = 5   # enum danse_fs_field (include/danse_mi355x.h)
FS_BCEND, FS_LEN, FS_POS, FS_IRSRC, FS_ZEND = range(FS_FIELDS)
# fewSamples device steps (enum danse_fs_step): one row (type, round, node
# mask, chunk-table row) per launch group
FS_STEP_CHUNK, FS_STEP_BCAST, FS_STEP_ZAN, FS_STEP_UPDATE = range(4)


def compile_rounds_fs(events, fs, p, nNodes: int, timeStamps, M) -> RoundTables:
    """Integer round tables for fewSamples broadcasts with ``efficientSpSBC``.

    Replays the reference events (``d_core.py:66-90``) with the state of
    ``broadcast`` (``d_classes.py:1043-1128``): the chunk size
    ``get_buffer_size_for_efficient_bc`` (``d_classes.py:1130-1160``: L times
    the whole number of L-blocks of node samples since the last broadcast),
    the T(z) IR refresh timer (``upTDfilterEvery``, ``d_classes.py:1090-1106``;
    no refresh at single-sensor nodes with ``noFusionAtSingleSensorNodes``) and
    the buffer flags of ``process_incoming_signals_buffers``
    (``d_classes.py:1701-1807``).  Every node stream is append-only, so the z
    frame an update consumes is the sender's stream[ZEND - N, ZEND) with ZEND
    the samples received so far (zero before 0, the reference's front
    padding).

    The broadcast instants of a node are its neighbours' update instants
    snapped to its own L-sample grid (``d_base.py:837-863``), so under SRO
    clocks a broadcast can fall anywhere between the updates: before the
    node's own update of the same iteration, after it (a faster node's chunk
    that its slower neighbour consumes in the same round, computed with the
    node's NEXT iteration's IR when the refresh timer fires there: L < 32 at
    200 ppm over 10 s), or twice in one iteration (L = Ns, the first
    snapped instants).  The device therefore runs a round as a list of steps
    (``fsSteps``): chunk appends (``fsEv`` rows: T(z) IR refresh + the currL
    convolution outputs per node), the round's analyses (``BCAST``: local
    frames, estimate synthesis and the z frames of the senders whose
    consumed chunks are in), late z-frame analyses (``ZAN``) and updates
    (``UPDATE``) of node subsets, in an order that respects every dependency
    of the reference's event order: a chunk after the update that wrote its
    IR source wExt[IRSRC], a z frame after the chunks it covers, an update
    after the z frames it consumes.  A plain round is CHUNK, BCAST, UPDATE.

    Accepted when in every round all receivers of a sender consume the same
    stream length (always true at K = 2 and on synchronous clocks).  Returns
    RoundTables with ``fsTab [R][K][FS_FIELDS]`` (ZEND per consuming round;
    the chunk fields of the round's first chunk of each node),
    ``fsEv [nEv][K][4]``, ``fsSteps [nSteps][4]``, ``fsRoundStep [R + 1]``
    and ``zStreamLen``."""
    if p.broadcastType != 'fewSamples':
        raise ValueError('compile_rounds_fs is for fewSamples broadcasts')
    if not p.efficientSpSBC:
        raise NotImplementedError('fewSamples without efficientSpSBC (one broadcast per L samples) on the device path')
    K, N, Ns = nNodes, p.DFTsize, p.Ns
    if K > 31:
        raise NotImplementedError('fewSamples device steps: node masks hold at most 31 nodes')
    Lb = int(p.broadcastLength)
    ts = [np.asarray(t, dtype=np.float64) for t in timeStamps]
    it = np.zeros(K, dtype=np.int64)              # iterations done per node
    lastBc = np.zeros(K)
    lastTD = np.zeros(K)
    streamLen = np.zeros(K, dtype=np.int64)
    buf = np.zeros((K, K), dtype=np.int64)
    chunks = [[] for _ in range(K)]               # per node, in order: [bcEnd, len, pos, irSrc]
    zEnd = {}                                     # (r, q) -> stream length consumed
    up = [[] for _ in range(K)]
    solve = [[] for _ in range(K)]
    tUp = [[] for _ in range(K)]
    flg = [[] for _ in range(K)]
    sync = True
    for ev in events:
        ks = list(ev.nodes)
        if ev.type != ['bc'] * K + ['up'] * K or ks != list(range(K)) * 2:
            sync = False
        for ii, (k, typ) in enumerate(zip(ks, ev.type)):
            k = int(k)
            if typ == 'bc':
                r = int(it[k])
                irSrc = -1
                if np.abs(ev.t - lastTD[k]) >= p.upTDfilterEvery:
                    if not (p.noFusionAtSingleSensorNodes and M[k] == 1):
                        irSrc = r
                    lastTD[k] = ev.t
                # sum((ts > last) & (ts <= t)) on the sorted clock
                n = int(np.searchsorted(ts[k], ev.t, 'right') - np.searchsorted(ts[k], lastBc[k], 'right'))
                currL = int(Lb * np.floor(n / Lb))
                lastBc[k] = ev.t
                if currL > N:
                    raise NotImplementedError(f'broadcast chunk of {currL} > N samples')
                chunks[k].append([int(np.floor(ev.t * fs[k])), currL, int(streamLen[k]), irSrc])
                streamLen[k] += currL
                for q in range(K):
                    if q != k:
                        buf[q, k] += currL
            else:
                r = int(it[k])
                up[k].append(int(np.floor(ev.t * fs[k])))
                solve[k].append(0 if ev.bypassUpdate[ii] else 1)
                tUp[k].append(ev.t)
                fr = np.zeros(K, dtype=np.int64)
                for q in range(K):
                    if q == k:
                        continue
                    Bq = buf[k, q]
                    if r == 0:
                        fr[q] = 0 if Bq == N else (-(N - Bq) if Bq < N else (Bq - N))
                    else:
                        if Bq > N:
                            raise NotImplementedError('more than N samples received between two updates')
                        fr[q] = 0 if Bq == Ns else (-(Ns - Bq) if Bq < Ns else (Bq - Ns))
                    if (r, q) in zEnd and zEnd[(r, q)] != streamLen[q]:
                        raise NotImplementedError('receivers of one sender consume different stream lengths')
                    zEnd[(r, q)] = int(streamLen[q])
                    buf[k, q] = 0
                flg[k].append(fr)
                it[k] += 1
    R = min(len(u) for u in up)
    if R < 1:
        raise ValueError('signal too short for one DANSE round')
    zTab = np.zeros((R, K), dtype=np.int64)
    for r in range(R):
        for q in range(K):
            # senders nobody consumed in a round keep the previous frame end
            zTab[r, q] = zEnd.get((r, q), zTab[r - 1, q] if r > 0 else 0)
    steps, evRows, roundStep, first = _fs_steps(chunks, zTab, K, R)
    tab = np.zeros((R, K, FS_FIELDS), dtype=np.int32)
    tab[:, :, FS_IRSRC] = -1
    for (r, k), (e, ln, pos, src) in first.items():
        tab[r, k, FS_BCEND], tab[r, k, FS_LEN], tab[r, k, FS_POS], tab[r, k, FS_IRSRC] = e, ln, pos, src
    tab[:, :, FS_ZEND] = zTab
    upEnd = np.array([u[:R] for u in up], dtype=np.int64).T
    # the broadcast kernel's phase 1 analyses "bcEnd" into the spectrum slot of
    # the next round's local frame: point it at upEnd[r + 1]
    bcEnd = np.empty_like(upEnd)
    bcEnd[:-1] = upEnd[1:]
    bcEnd[-1] = upEnd[-1]
    doSolve = np.array([x[:R] for x in solve], dtype=np.int32).T
    flags = np.stack([np.stack(f[:R]) for f in flg], axis=1)
    t = np.array([x[:R] for x in tUp], dtype=np.float64).T
    rt = RoundTables(bcEnd, upEnd, doSolve, R, t, np.zeros((R, K, K), np.uint8), flags, sync)
    rt.fsTab = tab
    rt.fsEv = evRows
    rt.fsSteps = steps
    rt.fsRoundStep = roundStep
    rt.fsChunks = [np.array(c, dtype=np.int64).reshape(-1, 4) for c in chunks]
    rt.zStreamLen = int(max(1, streamLen.max()))
    return rt


def _fs_steps(chunks, zTab, K, R):
    """List-schedules one round at a time (see ``compile_rounds_fs``).

    chunks[q]: node q's chunk events in stream order; zTab[r, q]: the stream
    length the round-r receivers of q consume.  Returns (steps [n][4] int32,
    chunk rows [nEv][K][4] int32, first step of each round [R + 1], {(r, k):
    the first chunk row of node k appended in round r})."""
    done = np.zeros(K, dtype=np.int64)     # updates done per node (wExt[done] is the newest)
    nxt = np.zeros(K, dtype=np.int64)      # next chunk event per node
    steps, rows, roundStep, first = [], [], [], {}
    full = (1 << K) - 1
    for r in range(R):
        roundStep.append(len(steps))
        pend = set(range(K))
        zdone = set()
        bcast = False
        while pend:
            progress = False
            # chunk steps: each node's next needed chunk (stream position below
            # what round r consumes) whose IR source wExt[IRSRC] is written
            while True:
                row = np.zeros((K, 4), dtype=np.int64)
                row[:, 3] = -1
                mask = 0
                for q in range(K):
                    c = chunks[q]
                    if nxt[q] < len(c) and c[nxt[q]][2] < zTab[r, q] and c[nxt[q]][3] <= done[q]:
                        row[q] = c[nxt[q]]
                        first.setdefault((r, q), tuple(c[nxt[q]]))
                        nxt[q] += 1
                        mask |= 1 << q
                if not mask:
                    break
                steps.append((FS_STEP_CHUNK, r, mask, len(rows)))
                rows.append(row)
                progress = True
            # z frames whose chunks are all in
            ready = 0
            for q in range(K):
                if q in zdone:
                    continue
                c = chunks[q]
                if nxt[q] >= len(c) or c[nxt[q]][2] >= zTab[r, q]:
                    ready |= 1 << q
                    zdone.add(q)
            if not bcast:
                steps.append((FS_STEP_BCAST, r, ready, -1))
                bcast = True
                progress = True
            elif ready:
                steps.append((FS_STEP_ZAN, r, ready, -1))
                progress = True
            # updates whose senders' z frames are analysed
            umask = 0
            for k in sorted(pend):
                if all(q in zdone for q in range(K) if q != k):
                    umask |= 1 << k
            if umask:
                steps.append((FS_STEP_UPDATE, r, umask, -1))
                for k in range(K):
                    if (umask >> k) & 1:
                        pend.discard(k)
                        done[k] = r + 1
                progress = True
            if not progress:
                raise NotImplementedError(f'fewSamples round {r}: no order of chunks, z frames and updates '
                                          'satisfies the event dependencies')
    roundStep.append(len(steps))
    st = np.array(steps, dtype=np.int32).reshape(-1, 4)
    ev = np.array(rows, dtype=np.int32).reshape(-1, K, 4)
    # (every update step of a plain round covers all nodes)
    assert full > 0
    return st, ev, np.array(roundStep, dtype=np.int32), first
