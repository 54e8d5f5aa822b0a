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


class ShardedRun:
    def __init__(self, engine, group=None):
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

    def exchange(self, r=0):
        i = r % self.slots
        self.dist.all_gather_into_tensor(self.slot[i], self.mine[i], group=self.group)

    def run(self, reset=True):
        e = self.eng
        if reset:
            e.reset()
        for r in range(e.R):
            e.bcast(r)
            self.exchange(r)
            e.update(r)
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

    def reset(self):
        from . import _lib as L
        L.check(self.e.lib.danse_engine_reset(self.e.eng, self.e.stream_ptr()), self.e.eng)

    def bcast(self, r):
        self.e.bcast(r)

    def update(self, r):
        self.e.update(r)

    def finish(self):
        self.e.finish()
