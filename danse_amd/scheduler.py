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
    """Per-round integer schedule for synchronous fully connected wholeChunk
    DANSE (every node broadcasts, then every node updates, once per round).

    bcEnd[r, k]   sample index one past the broadcast frame's end (floor(t fs))
    upEnd[r, k]   same for the update frame, already shifted by -(N - Ns)
    doSolve[r, k] 1 if the filter update is not bypassed (seq round robin)
    nRounds       number of rounds (= number of DANSE iterations per node)
    """
    bcEnd: np.ndarray
    upEnd: np.ndarray
    doSolve: np.ndarray
    nRounds: int
    t: np.ndarray = None        # [R] event instant of each round (float64)


def compile_rounds(events, fs, p, nNodes: int) -> RoundTables:
    """Checks that the schedule is round-synchronous (no SROs: all nodes share
    every instant, broadcasts before updates) and emits integer tables.
    Raises NotImplementedError otherwise (asynchronous clocks go through the
    per-event path)."""
    bcEnd, upEnd, doSolve, ts = [], [], [], []
    for ev in events:
        ks = list(ev.nodes)
        if ev.type != ['bc'] * nNodes + ['up'] * nNodes or ks != list(range(nNodes)) * 2:
            raise NotImplementedError('schedule is not round-synchronous (SROs or fewSamples)')
        if p.broadcastType != 'wholeChunk':
            raise NotImplementedError('fewSamples broadcasts use the per-event path')
        be = [int(np.floor(ev.t * fs[k])) for k in range(nNodes)]
        ue = [int(np.floor(ev.t * fs[k])) - (p.DFTsize - p.Ns) for k in range(nNodes)]
        bcEnd.append(be)
        upEnd.append(ue)
        doSolve.append([0 if b else 1 for b in ev.bypassUpdate[nNodes:]])
        ts.append(ev.t)
    return RoundTables(np.array(bcEnd, dtype=np.int64), np.array(upEnd, dtype=np.int64),
                       np.array(doSolve, dtype=np.int32), len(events), np.array(ts, dtype=np.float64))
