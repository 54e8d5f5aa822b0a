"""Node-sharded multi-process DANSE (danse_amd/dist.py) on CPU with gloo,
world size 2 and 4: every rank owns a node block, all-gathers the fused
spectra each round, and the per-node outputs equal the single-process run
bit for bit.  The compute is the float64 CPU stand-in (tests/_round_engine.py)
exposing the device engine's round/phase interface."""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _case(sro=False):
    from golden_cases import BATTERY, _d
    c = dict(name='dist', M=[2, 2, 2, 2], dur=1.6, seed=21, danse=_d(BATTERY, nodeUpdating='asy'))
    if sro:
        c['sros'] = [0.0, 150.0, 300.0, 450.0]
    return c


def _setup(case, nodes=None):
    from _util import make_case_params
    from danse_amd.scene import make_scene
    dp, wp = make_case_params(case)
    scenes = []
    for sd in (case['seed'], case['seed'] + 1):
        sc = make_scene(case['M'], sigDur=case['dur'], seed=sd, nodes=nodes, SROperNode=case.get('sros'))
        sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
        scenes.append(sc)
    return dp, scenes


def _worker(rank, world, port, outdir, sro=False):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / 'tests'))
    sys.path.insert(0, str(ROOT / 'tests' / 'golden'))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from danse_amd.dist import ShardedRun, node_range
    from _round_engine import RoundEngine
    case = _case(sro)
    k0, k1 = node_range(len(case['M']), world, rank)
    dp, scenes = _setup(case, nodes=list(range(k0, k1)))
    eng = RoundEngine(scenes, dp, nodeRange=(k0, k1))
    ShardedRun(eng).run()
    for s in range(eng.S):
        for k in range(k0, k1):
            np.save(Path(outdir) / f'd_{s}_{k}.npy', eng.st[s][k]['d'])
            np.save(Path(outdir) / f'w_{s}_{k}.npy', eng.st[s][k]['w'])
    dist.barrier()
    dist.destroy_process_group()


def _single(sro=False):
    from _round_engine import RoundEngine
    dp, scenes = _setup(_case(sro))
    eng = RoundEngine(scenes, dp)
    eng.set_zspec(torch.zeros(eng.zspec_numel(), dtype=torch.float32))
    eng.reset()
    for r in range(eng.R):
        eng.bcast(r)
        eng.update(r)
    return eng, dp, scenes


@pytest.mark.parametrize('world,sro', [(2, False), (4, False), (2, True)], ids=['w2', 'w4', 'w2_sro'])
def test_node_sharded_equals_single_process(world, sro):
    """sro: SRO clocks (0/150/300/450 ppm), two exchanged round slots and
    receivers reading the previous round's slot (zLag)."""
    ref, _, _ = _single(sro)
    if sro:
        assert not ref.rt.synchronous and ref.zspec_slots == 2 and int(ref.rt.zLag.max()) == 1
    with tempfile.TemporaryDirectory() as td:
        port = 29500 + (os.getpid() % 1000) + world + (7 if sro else 0)
        mp.spawn(_worker, args=(world, port, td, sro), nprocs=world, join=True)
        for s in range(ref.S):
            for k in range(ref.K):
                d = np.load(Path(td) / f'd_{s}_{k}.npy')
                w = np.load(Path(td) / f'w_{s}_{k}.npy')
                assert np.array_equal(d, ref.st[s][k]['d']), (s, k)
                assert np.array_equal(w, ref.st[s][k]['w']), (s, k)


def test_round_engine_matches_oracle():
    """The stand-in reproduces the oracle (up to the complex64 spectra buffer)."""
    from oracle import danse_ref_cpu as O
    eng, dp, scenes = _single()
    for s, sc in enumerate(scenes):
        ov = O.danse(sc, dp, vadMinProp=0.5)
        d = np.stack([eng.st[s][k]['d'] for k in range(eng.K)], axis=1)
        err = np.max(np.abs(d - ov.d)) / np.max(np.abs(ov.d))
        assert err < 1e-4, err


def _worker_subgroups(rank, world, port, outdir):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / 'tests'))
    sys.path.insert(0, str(ROOT / 'tests' / 'golden'))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from danse_amd.dist import ShardedRun, control_group, node_range
    from _round_engine import RoundEngine
    # two independent runs on the sub-groups {0, 1} and {2, 3} (every rank
    # creates both groups, as new_group requires)
    groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
    mine = groups[rank // 2]
    sub = rank % 2
    case = _case()
    k0, k1 = node_range(len(case['M']), 2, sub)
    dp, scenes = _setup(case, nodes=list(range(k0, k1)))
    eng = RoundEngine(scenes, dp, nodeRange=(k0, k1))
    run = ShardedRun(eng, group=mine)
    assert run.world == 2 and run.rank == sub
    run.run()
    # the RCCL-side control group: over this sub-group's ranks only, created
    # by its members alone; a failing verdict on rank 3 stays inside {2, 3}
    ctl = control_group(mine, 'nccl')
    t = torch.tensor([0 if rank == 3 else 1], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctl)
    np.save(Path(outdir) / f'verdict_{rank}.npy', t.numpy())
    for s in range(eng.S):
        for k in range(k0, k1):
            np.save(Path(outdir) / f'd_{rank // 2}_{s}_{k}.npy', eng.st[s][k]['d'])
    dist.barrier()
    dist.destroy_process_group()


def test_subgroup_runs_and_control_groups():
    """World size 4 as two sub-groups of 2: each sub-group's
    ShardedRun equals the single-process run, and the control group of a
    sub-group (dist.control_group, what an RCCL run uses for its gate
    verdicts) only spans that sub-group's ranks."""
    ref, _, _ = _single()
    with tempfile.TemporaryDirectory() as td:
        port = 29500 + (os.getpid() % 1000) + 31
        mp.spawn(_worker_subgroups, args=(4, port, td), nprocs=4, join=True)
        verd = [int(np.load(Path(td) / f'verdict_{r}.npy')[0]) for r in range(4)]
        assert verd == [1, 1, 0, 0], verd
        for g in range(2):
            for s in range(ref.S):
                for k in range(ref.K):
                    assert np.array_equal(np.load(Path(td) / f'd_{g}_{s}_{k}.npy'), ref.st[s][k]['d']), (g, s, k)


class _SegEngine:
    """Protocol stand-in for fewSamples rounds whose updates run as several
    node-subset steps (DanseEngine.update_segments): on odd rounds the first
    half of the nodes updates first and each of them then writes a late z
    value (the late chunk's z frame), which the second half's update must
    read -- on another rank only if ShardedRun exchanges before segment 1."""
    R, K = 6, 4

    def __init__(self, k0, k1):
        self.k0, self.k1 = k0, k1
        self.zspec_slots = 1
        self.torch_device = 'cpu'

    def zspec_numel(self):
        return self.K

    def set_zspec(self, t):
        self.z = t

    def reset(self):
        self.seen = {}

    def bcast(self, r):
        for k in range(self.k0, self.k1):
            self.z[k] = 100.0 * r + k

    def update_segments(self, r):
        return 2 if r % 2 else 1

    def segment_nodes(self, r, j):
        h = self.K // 2
        return set(range(h)) if j == 0 else set(range(h, self.K))

    def update(self, r, seg=None):
        nodes = set(range(self.K)) if seg is None else self.segment_nodes(r, seg)
        for k in sorted(nodes & set(range(self.k0, self.k1))):
            self.seen[(r, k)] = self.z.clone().numpy()
        if seg == 0:
            for k in sorted(nodes & set(range(self.k0, self.k1))):
                self.z[k] = 100.0 * r + k + 0.5

    def finish(self):
        pass


def _worker_segments(rank, world, port, outdir):
    sys.path.insert(0, str(ROOT))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from danse_amd.dist import ShardedRun, node_range
    k0, k1 = node_range(_SegEngine.K, world, rank)
    eng = _SegEngine(k0, k1)
    ShardedRun(eng).run()
    for (r, k), v in eng.seen.items():
        np.save(Path(outdir) / f'seen_{r}_{k}.npy', v)
    dist.barrier()
    dist.destroy_process_group()


def test_split_round_segments_exchange_late_z():
    """Node-sharded split rounds (fewSamples, SRO clocks with L < Ns): the
    nodes of a later update segment see the late z values the earlier
    segment's nodes wrote on the other rank, as in the single-process run."""
    ref = _SegEngine(0, _SegEngine.K)
    ref.set_zspec(torch.zeros(ref.zspec_numel()))
    ref.reset()
    for r in range(ref.R):
        ref.bcast(r)
        n = ref.update_segments(r)
        for j in range(n):
            ref.update(r, j if n > 1 else None)
    assert np.array_equal(ref.seen[(1, 3)], [100.5, 101.5, 102, 103])
    with tempfile.TemporaryDirectory() as td:
        port = 29500 + (os.getpid() % 1000) + 43
        mp.spawn(_worker_segments, args=(2, port, td), nprocs=2, join=True)
        for (r, k), v in ref.seen.items():
            assert np.array_equal(np.load(Path(td) / f'seen_{r}_{k}.npy'), v), (r, k)
