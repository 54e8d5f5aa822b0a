"""Multi-GPU DANSE: one process per GPU, nodes sharded over ranks.

SURVEY §8e: the online engine shards by node; the only exchange per frame is
the fused-signal broadcast (``fill_buffers``, ``danse_toolbox/d_classes.py:
1185-1224``), which becomes ONE in-place all-gather per round of the fused
spectra of every node (RCCL over xGMI on MI355X; gloo on CPU for tests).
Each rank runs the broadcast phase for the nodes it owns, the all-gather
completes the node-major ``[K][S][F]`` spectra buffer on every rank, then each
rank runs the update phase of its nodes.  No other data-path collective.

``ShardedRun`` drives any engine exposing ``R, K, k0, k1, reset(), bcast(r),
update(r), finish(), zspec_numel(), set_zspec(tensor)`` (the HIP engine
wrapper ``ShardedEngine`` below, or a CPU stand-in in the tests).
"""
from __future__ import annotations

import ctypes


def node_range(K: int, world: int, rank: int):
    """Contiguous, equal node blocks (the all-gather needs equal chunks)."""
    if K % world != 0:
        raise ValueError(f'K={K} nodes cannot be split evenly over {world} ranks')
    per = K // world
    return rank * per, (rank + 1) * per


def control_group(group, backend):
    """The group the host-side control traffic of a run over ``group`` uses.

    Over RCCL it is a gloo group of the SAME ranks as ``group`` (an RCCL
    collective issued outside a captured graph on the graph's communicator
    makes later replays diverge, ``profiles/round3/rccl_graph_mixing_r3d.log``);
    for a sub-group only its members create it (local synchronization), so
    other shards neither take part nor see its verdicts.  Over gloo it is
    ``group`` itself."""
    import torch.distributed as dist
    if str(backend).lower() != 'nccl':
        return group
    if group is None or group is dist.group.WORLD:
        return dist.new_group(backend='gloo')
    return dist.new_group(ranks=dist.get_process_group_ranks(group), backend='gloo',
                          use_local_synchronization=True)


class ShardedRun:
    """Drives a node-sharded engine over ``torch.distributed``.

    Per round r: ``bcast(r)`` for the owned nodes, the in-place all-gather of
    the fused spectra, the start gate of round r for the owned nodes, then
    ``update(r)`` -- or, for a fewSamples round whose updates run as several
    node-subset steps (``update_segments(r)`` > 1), ``update(r, j)`` per
    segment with one more all-gather before each segment after the first.

    The reference's start gate (``check_covariance_matrices``,
    ``d_classes.py:1430-1540``) decides when each node starts updating from
    its own SCMs only, so each rank checks its own nodes.  A delayed start
    changes that node's filters and, through z, every other rank's results,
    so the ranks agree on one outcome: the run goes speculatively first (the
    flags assume every check passes; the checks run inside the run), the
    per-rank verdicts are all-reduced (MIN), and if any rank saw a failure
    every rank repeats the run exactly, deciding each candidate's start
    synchronously at its round (as ``DanseEngine._run_gated``).

    With RCCL the speculative (or ungated) round sequence -- reset, 310 x
    (bcast, all-gather, gate, update), finish -- is captured once into a CUDA
    graph and replayed (``graph=None``: on when the backend is nccl).  With
    gloo and device tensors the exchange is staged through host memory.
    """

    def __init__(self, engine, group=None, graph=None, ctl=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        k0, k1 = node_range(engine.K, self.world, self.rank)
        if (k0, k1) != (engine.k0, engine.k1):
            raise ValueError('engine node range does not match this rank')
        n = engine.zspec_numel()
        self.zbuf = torch.zeros(n, dtype=torch.float32, device=engine.torch_device)
        engine.set_zspec(self.zbuf)
        # the HIP engine keeps two round slots ([2][K][S][F], round r -> slot
        # r & 1) so that SRO-lagged receivers can read the previous round
        self.slots = getattr(engine, 'zspec_slots', 1)
        per = n // self.slots
        chunk = per // self.world
        self.slot = [self.zbuf[i * per:(i + 1) * per] for i in range(self.slots)]
        self.mine = [v[self.rank * chunk:(self.rank + 1) * chunk] for v in self.slot]
        backend = str(dist.get_backend(group)).lower()
        # gloo cannot gather device tensors in place: stage through the host
        self.stage = backend == 'gloo' and self.zbuf.device.type != 'cpu'
        if self.stage:
            self.hslot = [torch.zeros(per, dtype=torch.float32) for _ in range(self.slots)]
        # node-sharded DXCP-PhaT: the Ns new z samples of every node per round
        # ([K][S][Ns], this rank's nodes one chunk) for the receivers' estimators
        nz = engine.zchunk_numel() if getattr(engine, 'zchunk_numel', None) is not None else 0
        self.zc = None
        if nz > 0:
            self.zc = torch.zeros(nz, dtype=torch.float32, device=engine.torch_device)
            engine.set_zchunk(self.zc)
            zper = nz // self.world
            self.zc_mine = self.zc[self.rank * zper:(self.rank + 1) * zper]
            if self.stage:
                self.zc_host = torch.zeros(nz, dtype=torch.float32)
        self.graph = (backend == 'nccl') if graph is None else bool(graph)
        # host-side control traffic (gate verdicts, callers' barriers)
        self.ctl = ctl if ctl is not None else control_group(group, backend)
        self._graphs = {}
        self._graph_gen = None
        self._eager_runs = 0

    def exchange(self, r=0):
        i = r % self.slots
        # (issued at world size 1 too: an identity, but a real collective in
        # the captured round graph, which test_rccl_graph_captured_rounds
        # replays)
        if self.stage:
            mine = self.mine[i].cpu()
            self.dist.all_gather_into_tensor(self.hslot[i], mine, group=self.group)
            self.slot[i].copy_(self.hslot[i])
            if self.zc is not None:
                self.dist.all_gather_into_tensor(self.zc_host, self.zc_mine.cpu(), group=self.group)
                self.zc.copy_(self.zc_host)
        else:
            self.dist.all_gather_into_tensor(self.slot[i], self.mine[i], group=self.group)
            if self.zc is not None:
                self.dist.all_gather_into_tensor(self.zc, self.zc_mine, group=self.group)
        if self.zc is not None:
            self.eng.unpack_zchunk(r)

    def _rounds(self, reset, gate):
        e = self.eng
        if reset:
            e.reset()
        for r in range(e.R):
            e.bcast(r)
            self.exchange(r)
            if gate:
                e.gate_launch(r)
            self._update(r)
        e.finish()

    def _nseg(self, r):
        f = getattr(self.eng, 'update_segments', None)
        return 1 if f is None else f(r)

    def _update(self, r, pending=None):
        """The update phase of round r: one call, or (a fewSamples round
        whose updates run as several node-subset steps) one segment per
        update step with an exchange before every segment after the first
        (its senders' late z frames were analysed in the previous one); the
        exact gate decides each segment's nodes right before it."""
        e = self.eng
        n = self._nseg(r)
        for j in range(n):
            if j:
                self.exchange(r)
            if pending is not None and pending and min(pending.values()) == r:
                if n == 1:
                    e.gate_decide(r, pending)
                else:
                    e.gate_decide(r, pending, nodes=e.segment_nodes(r, j))
            if n == 1:
                e.update(r)
            else:
                e.update(r, j)

    def _sequence(self, reset, gate):
        """The round sequence, eagerly or as a replayed CUDA graph (captured
        on the second call, once the communicator and the kernels are warm)."""
        torch = self.torch
        key = (bool(reset), bool(gate))
        if not self.graph or self.stage or self.zbuf.device.type == 'cpu':
            return self._rounds(reset, gate)
        # a captured graph holds the engine's flag-derived launch sizes and
        # gate buffer pointers: drop it when the engine's flags or gate
        # schedule changed since the capture
        gen = getattr(self.eng, 'graph_gen', None)
        if gen != self._graph_gen:
            self._graphs.clear()
            self._graph_gen = gen
        g = self._graphs.get(key)
        if g is None:
            if self._eager_runs < 1:
                self._eager_runs += 1
                return self._rounds(reset, gate)
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(device=self.zbuf.device)
            side.wait_stream(torch.cuda.current_stream(self.zbuf.device))
            # the state reset (memsets + two kernels) stays OUT of the graph:
            # captured, its memset nodes were not re-applied from the second
            # replay on (the second replay started from the previous run's
            # streams and estimates: profiles/round3/pytest_gpu_r3g.log)
            with torch.cuda.graph(g, stream=side):
                self._rounds(False, gate)
            self._graphs[key] = g
        if reset:
            self.eng.reset()
        g.replay()

    def _all_ok(self, ok):
        gloo = self.ctl is not self.group or self.zbuf.device.type == 'cpu' or self.stage
        t = self.torch.tensor([1 if ok else 0], dtype=self.torch.int32, device='cpu' if gloo else self.zbuf.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.ctl)
        return bool(int(t.item()))

    def barrier(self):
        """A barrier that leaves the captured RCCL rounds intact (gloo)."""
        self.dist.barrier(group=self.ctl)

    def run(self, reset=True, gate=True):
        e = self.eng
        gating = getattr(e, 'gating', None) is not None and e.gating(gate)
        if not gating:
            if getattr(e, 'begin_run', None) is not None:
                # the same bookkeeping as a gated run: init slots re-loaded,
                # counter-compiled flags restored, no in-run gate
                e.begin_run(speculative=False)
            self._sequence(reset, False)
            return self
        if not e.gate_spec_failed:
            e.begin_run(speculative=True)
            self._sequence(reset, True)
            if self._all_ok(e.gate_ok()):
                return self
            # some rank's speculative start was wrong: every rank repeats
            e.mark_gate_failed()
        e.begin_run(speculative=False)
        e.reset()
        pending = e.gate_pending()
        for r in range(e.R):
            e.bcast(r)
            self.exchange(r)
            self._update(r, pending)
        e.finish()
        return self


class ShardedEngine:
    """Adapter of ``danse_amd.engine.DanseEngine`` to the ShardedRun interface."""

    def __init__(self, engine):
        self.e = engine
        self.R, self.K, self.k0, self.k1 = engine.R, engine.K, engine.k0, engine.k1
        self.torch_device = f'cuda:{engine.device}'
        self.zspec_slots = 2

    def zspec_numel(self):
        _, nb = self.e.zspec()
        return nb // 4

    def set_zspec(self, t):
        from . import _lib as L
        L.check(self.e.lib.danse_engine_set_zspec(self.e.eng, ctypes.c_void_p(t.data_ptr())), self.e.eng)

    def zchunk_numel(self):
        """DXCP-PhaT on a node-sharded engine: [K][S][Ns] floats of z chunks
        to exchange per round (0 otherwise)."""
        e = self.e
        if not getattr(e, 'dxcp', False) or (e.k0, e.k1) == (0, e.K):
            return 0
        return e.K * e.S * e.Ns

    def set_zchunk(self, t):
        from . import _lib as L
        L.check(self.e.lib.danse_engine_set_zchunk(self.e.eng, ctypes.c_void_p(t.data_ptr())), self.e.eng)

    def unpack_zchunk(self, r):
        from . import _lib as L
        L.check(self.e.lib.danse_engine_unpack_zchunk(self.e.eng, int(r), self.e.stream_ptr()), self.e.eng)

    def reset(self):
        from . import _lib as L
        L.check(self.e.lib.danse_engine_reset(self.e.eng, self.e.stream_ptr()), self.e.eng)

    def bcast(self, r):
        self.e.bcast(r)

    def update(self, r, seg=None):
        self.e.update(r, seg)

    def update_segments(self, r):
        return self.e.update_segments(r)

    def segment_nodes(self, r, seg):
        return self.e.segment_nodes(r, seg)

    def finish(self):
        self.e.finish()

    @property
    def graph_gen(self):
        """Changes whenever the engine's flags or gate schedule do."""
        return self.e.graph_gen

    # the start gate (DanseEngine's caller-sequenced gate API)
    def gating(self, gate=True):
        return self.e.gating(gate)

    def begin_run(self, speculative):
        return self.e.begin_run(speculative)

    def gate_launch(self, r):
        self.e.gate_launch(r)

    def gate_ok(self):
        return self.e.gate_ok()

    def mark_gate_failed(self):
        self.e.mark_gate_failed()

    @property
    def gate_spec_failed(self):
        return self.e.gate_spec_failed

    def gate_pending(self):
        return self.e.gate_pending()

    def gate_decide(self, r, pending, nodes=None):
        self.e.gate_decide(r, pending, nodes=nodes)
