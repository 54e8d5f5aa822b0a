"""Node-sharded batch DANSE exchange protocol (danse_amd/batch.py
run_node_sharded + allgather_exchange) on CPU with gloo, world size 2 and 3.
The engine is a CPU stand-in with the device engine's run_iters / pack_wext /
unpack_wext interface: iteration it computes, for its own nodes only, a new
external filter from EVERY node's previous one (as batch z couples all
nodes), so any missing, stale or misplaced exchange changes the result.  The
per-node histories must equal a single-process run of all nodes bit for bit.
The device side of the same protocol is test_gpu_parity.py::
test_batch_node_sharded_equals_full."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent
K, S, F, MMAX, ITERS = 5, 2, 3, 2, 4


class _FakeBatch:
    def __init__(self, k0, k1):
        self.torch = torch
        self.S, self.K, self.F, self.Mmax, self.iters = S, K, F, MMAX, ITERS
        self.k0, self.k1 = k0, k1
        rng = np.random.default_rng(3)
        self.M = [1 + (k % MMAX) for k in range(K)]
        self.wExt = np.zeros((K, ITERS + 1, S, F, MMAX), dtype=np.complex64)
        for k in range(K):
            self.wExt[k, 0, :, :, :self.M[k]] = rng.standard_normal((S, F, self.M[k]))
        self.wExt[:, 1:] = np.nan   # never read before written / received

    def wext_chunk(self):
        return self.F * self.Mmax

    def run_iters(self, it0, it1, stream=None):
        for it in range(it0, it1):
            z = self.wExt[:, it].sum(axis=(0, 3))          # needs every node's slot it
            assert np.all(np.isfinite(z)), 'stale external filter read'
            for k in range(self.k0, self.k1):
                nxt = 0.5 * self.wExt[k, it] + (0.1 * (k + 1)) * z[:, :, None]
                nxt[:, :, self.M[k]:] = 0
                self.wExt[k, it + 1] = nxt

    def pack_wext(self, slot, out, stream=None):
        n = (self.k1 - self.k0) * S * F * MMAX
        out[:n] = torch.from_numpy(self.wExt[self.k0:self.k1, slot].reshape(-1).copy())

    def unpack_wext(self, slot, src, stream=None):
        g = src[:K * S * F * MMAX].numpy().reshape(K, S, F, MMAX)
        for k in range(K):
            if not self.k0 <= k < self.k1:
                self.wExt[k, slot] = g[k]


def _worker(rank, world, port, outdir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from danse_amd.batch import node_ranges, run_node_sharded, allgather_exchange
    rngs, c = node_ranges(K, world)
    eng = _FakeBatch(*rngs[rank])
    run_node_sharded(eng, allgather_exchange(dist, world), c, device='cpu')
    np.save(os.path.join(outdir, f'r{rank}.npy'), eng.wExt)
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_batch_node_sharded_protocol_gloo(world, tmp_path):
    from danse_amd.batch import node_ranges
    full = _FakeBatch(0, K)
    full.run_iters(0, ITERS)
    port = 29600 + world + (os.getpid() % 500)
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    rngs, _ = node_ranges(K, world)
    for r in range(world):
        w = np.load(tmp_path / f'r{r}.npy')
        assert np.array_equal(w, full.wExt), r    # own nodes computed, others received


def test_node_ranges():
    from danse_amd.batch import node_ranges
    assert node_ranges(5, 2) == ([(0, 3), (3, 5)], 3)
    assert node_ranges(32, 8)[0][-1] == (28, 32)
    with pytest.raises(ValueError):
        node_ranges(4, 3)   # blocks of 2: the third rank would own nothing
