"""Node-sharded online DANSE with the HIP engine in separate processes
(``danse_amd.dist.ShardedRun`` over ``DanseEngine``, ``-m gpu``):

* world size 2 over gloo, both ranks on cuda:0, the fused-spectra all-gather
  staged through host memory: each rank owns half the nodes and the owned
  nodes' outputs equal the single-engine run bit for bit, including
  - a start the reference gate delays (``check_covariance_matrices``,
    ``d_classes.py:1430-1540``): the speculative run fails on one rank, the
    verdicts are all-reduced and every rank repeats the run exactly;
  - CohDrift SRO estimation on a sharded engine (each rank estimates for its
    own receivers from the all-gathered fused spectra);
  - fewSamples rounds split into node-subset update steps (one more
    all-gather per extra step) with centralised / SSBC estimates;
* world size 1 over RCCL: the round sequence (bcast, the in-place RCCL
  all-gather of the fused spectra -- an identity at one rank, but a real
  collective in the graph --, gate, update) captured into a CUDA graph and
  replayed equals the eager run.
"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent

from golden_cases import BATTERY, _d  # noqa: E402

CASES = {
    # the start gate delays nodes 0, 2, 3 (oracle starts [54, 27, 29, 28],
    # counters allow 27 everywhere)
    'gate_delay_k4': dict(name='gate_delay_k4', M=[2, 2, 2, 2], dur=3.0, seed=5,
                          danse=_d(BATTERY, nodeUpdating='asy', covMatInitType='eye_and_random',
                                   covMatRandomInitScaling=1e-6, use1stFrameAsBasis=False, t_expAvg50p=0.1)),
    'cohdrift_k4': dict(name='cohdrift_k4', M=[2, 3, 2, 2], dur=3.0, seed=15, sros=[0, 60, 120, 180],
                        danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=True, includeFSDflags=True,
                                 estimateSROs='CohDrift', cohDrift=dict(estimationMethod='ls'))),
    'plain_k4': dict(name='plain_k4', M=[3, 3, 3, 3], dur=2.0, seed=2, danse=_d(BATTERY, nodeUpdating='asy')),
    # DXCP-PhaT per (receiver, sender) on a node-sharded engine: the senders
    # of the other rank reach the receivers' estimators through the per-round
    # z-chunk all-gather (long enough for the estimators' first outputs)
    'dxcp_k4': dict(name='dxcp_k4', M=[2, 2, 2, 2], dur=7.0, seed=16, sros=[0, 60, 120, 180],
                    danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=True, includeFSDflags=True,
                             estimateSROs='DXCPPhaT')),
    # fewSamples with split rounds (L = 8 at 200 ppm: round 94's updates run
    # as two node-subset steps, one more all-gather between them) and the
    # centralised / SSBC families (each rank analyses the other's raw frames)
    'fs_split_centr_k2': dict(name='fs_split_centr_k2', M=[2, 3], dur=4.0, seed=0, sros=[0.0, 200.0],
                              danse=_d(BATTERY, nodeUpdating='asy', broadcastType='fewSamples', broadcastLength=8,
                                       computeCentralised=True, computeSingleSensorBroadcast=True,
                                       compensateSROs=False)),
}


def _setup(case):
    from _util import make_case_params, make_case_scene
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    return sc, dp, wp


def _save(dv, k0, k1, outdir, tag):
    for k in range(k0, k1):
        np.save(Path(outdir) / f'{tag}_d_{k}.npy', dv.d[:, k])
        np.save(Path(outdir) / f'{tag}_w_{k}.npy', dv.wTilde[k])
        np.save(Path(outdir) / f'{tag}_e_{k}.npy', dv.wTildeExt[k])
        np.save(Path(outdir) / f'{tag}_s_{k}.npy', np.asarray(dv.startRound[k]))
        for nm in ('dCentr', 'dSSBC'):
            if getattr(dv, nm, None) is not None:
                np.save(Path(outdir) / f'{tag}_{nm}_{k}.npy', getattr(dv, nm)[:, k])
        if getattr(dv, 'SROsEstimates', None) is not None:
            np.save(Path(outdir) / f'{tag}_sro_{k}.npy', np.asarray(dv.SROsEstimates[k]))


def _worker(rank, world, port, outdir, name, backend, passes):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / 'tests'))
    sys.path.insert(0, str(ROOT / 'tests' / 'golden'))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    if backend == 'nccl':
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda:0'))
    else:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    from danse_amd.dist import ShardedRun, ShardedEngine, node_range
    from danse_amd.engine import DanseEngine
    case = CASES[name]
    sc, dp, wp = _setup(case)
    k0, k1 = node_range(len(case['M']), world, rank)
    eng = DanseEngine([sc], dp, nodeRange=(k0, k1))
    run = ShardedRun(ShardedEngine(eng))
    for i in range(passes):
        run.run(reset=True)
        torch.cuda.synchronize()
        _save(eng.outputs()[0], k0, k1, outdir, f'p{i}')
    np.save(Path(outdir) / f'graphs_{rank}.npy', np.array(len(run._graphs)))
    np.save(Path(outdir) / f'specfail_{rank}.npy', np.array(int(eng.gate_spec_failed)))
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def _spawn(name, world, backend, passes):
    import torch.multiprocessing as mp
    from danse_amd.core import danse_multi
    case = CASES[name]
    sc, dp, wp = _setup(case)
    ref = danse_multi([sc], dp)[0]
    td = tempfile.mkdtemp(prefix='danse_dist_')
    port = 29600 + (os.getpid() % 500) + 3 * world + (1 if backend == 'nccl' else 0)
    mp.spawn(_worker, args=(world, port, td, name, backend, passes), nprocs=world, join=True)
    return ref, Path(td)


def _compare(ref, td, K, passes):
    # diagnostics first (an intermittent pass-2 mismatch of d was seen once,
    # gpurun_out/pytest_gpu_r3h.log): which outputs differ and by how much
    for i in range(passes):
        for k in range(K):
            dd = np.max(np.abs(np.load(td / f'p{i}_d_{k}.npy') - ref.d[:, k]))
            dw = np.max(np.abs(np.load(td / f'p{i}_w_{k}.npy') - ref.wTilde[k]))
            de = np.max(np.abs(np.load(td / f'p{i}_e_{k}.npy') - ref.wTildeExt[k]))
            if dd or dw or de:
                print(f'pass {i} node {k}: max |d| diff {dd:.3e}, |w| {dw:.3e}, |wExt| {de:.3e}', flush=True)
    for i in range(passes):
        for k in range(K):
            assert np.array_equal(np.load(td / f'p{i}_d_{k}.npy'), ref.d[:, k]), (i, k)
            assert np.array_equal(np.load(td / f'p{i}_w_{k}.npy'), ref.wTilde[k]), (i, k)
            assert np.array_equal(np.load(td / f'p{i}_e_{k}.npy'), ref.wTildeExt[k]), (i, k)
            assert int(np.load(td / f'p{i}_s_{k}.npy')) == int(ref.startRound[k]), (i, k)
            for nm in ('dCentr', 'dSSBC'):
                f = td / f'p{i}_{nm}_{k}.npy'
                if getattr(ref, nm, None) is not None:
                    assert np.array_equal(np.load(f), getattr(ref, nm)[:, k]), (i, nm, k)
            f = td / f'p{i}_sro_{k}.npy'
            if f.exists() and getattr(ref, 'SROsEstimates', None) is not None:
                assert np.array_equal(np.load(f), np.asarray(ref.SROsEstimates[k])), (i, k)


@pytest.mark.parametrize('name', ['gate_delay_k4', 'cohdrift_k4', 'dxcp_k4', 'fs_split_centr_k2'])
def test_sharded_processes_match_single_engine(name):
    ref, td = _spawn(name, 2, 'gloo', 2)
    K = len(CASES[name]['M'])
    if name == 'gate_delay_k4':
        # the gate really delays: the starts differ from the counter rounds
        assert sorted(int(x) for x in ref.startRound) == [27, 28, 29, 54], ref.startRound
        assert int(np.load(td / 'specfail_0.npy')) == 1 and int(np.load(td / 'specfail_1.npy')) == 1
    _compare(ref, td, K, 2)
    if name == 'dxcp_k4':
        # the estimates reached the compensation on both ranks
        for k in range(K):
            assert np.count_nonzero(np.load(td / f'p0_sro_{k}.npy')) > 0, k


@pytest.mark.parametrize('name', ['plain_k4', 'gate_delay_k4'])
def test_rccl_graph_captured_rounds(name):
    """RCCL, world size 1: pass 0 eager, pass 1 captures the rounds (R
    in-graph all-gathers) into a CUDA graph and replays it, passes 2 and 3
    replay it again (speculative gate inside the graph): three replays
    bit-equal to the single engine; the gate-delay case falls back to the
    exact host-gated loop."""
    ref, td = _spawn(name, 1, 'nccl', 4)
    _compare(ref, td, len(CASES[name]['M']), 4)
    if name == 'plain_k4':
        assert int(np.load(td / 'graphs_0.npy')) == 1
