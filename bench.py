#!/usr/bin/env python3
"""DANSE frame-update throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scenes S] [--shard nodes|scenes]

Workload (BASELINE.json configs[1], "B"): GEVD-DANSE rank 1, fully connected
K = 8 nodes x 4 mics, N_STFT = 1024 (513 bins), asynchronous node updating,
battery settings (config_files/sandbox_config_battery20230919.yaml), 10 s
synthetic random-IR scenes at 16 kHz (310 DANSE rounds).  A "step" is one
full pass of the online engine over one batch of S independent scenes per GPU
(state reset + every round: WOLA analysis, compression, z synthesis, SCM
update, GEVD filter update, external filters, estimate synthesis), inputs
resident in HBM.  value = node x bin frame-updates / s over the whole job.

Multi-GPU (one process per GPU, torchrun): --shard nodes (default) splits the
K nodes of every scene over the ranks and all-gathers the fused-signal
spectra every round over RCCL (the per-frame broadcast of DANSE); the batch
holds S scenes per GPU (weak scaling).  --shard scenes runs independent
scene replicas (no collective).

Also reported: the roofline of the dominant kernel (update_kernel) from live
HIP-event timing, its HBM traffic from two rocprofv3 PMC passes
(FETCH_SIZE x2 + WRITE_SIZE, run as child processes), and the CPU oracle (a
float64 NumPy restatement of the reference algorithm, "port") timed on this
host on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md, chip-level parameters


def _battery_params(M, nodeUpdating='asy', **extra):
    from danse_amd import params as P
    dp = P.DANSEparameters(simType='online', nodeUpdating=nodeUpdating, performGEVD=True, GEVDrank=1, **extra,
                           use1stFrameAsBasis=True, filterInitType='selectFirstSensor',
                           forcedBetaExternalFilters=0.7, t_expAvg50p=1, t_expAvg50pExternalFilters=1,
                           noFusionAtSingleSensorNodes=True, startComputeMetricsAt='after_5s')
    wp = P.WASNparameters(trueRoom=False, signalType='random', nSensorPerNode=list(M), sigDur=10,
                          VADenergyDecrease_dB=40, VADwinLength=0.04, vadMinProportionActive=0.25,
                          snr=5, selfnoiseSNR=15,
                          topologyParams=P.TopologyParameters(topologyType='fully-connected', seed=12348))
    wp.__post_init__()
    dp.__post_init__()
    dp.get_wasn_info(wp)
    return dp, wp


WORKLOADS = {
    # BASELINE.json configs[1]
    'B': dict(M=[4] * 8, dur=10.0, nodeUpdating='asy', desc='B: GEVD-DANSE r1, K=8 x 4 mics, N=1024, asy, 10 s'),
    'B_seq': dict(M=[4] * 8, dur=10.0, nodeUpdating='seq', desc='B (seq): GEVD-DANSE r1, K=8 x 4 mics, seq, 10 s'),
    'small': dict(M=[2] * 4, dur=3.0, nodeUpdating='asy', desc='small smoke workload K=4 x 2, 3 s'),
    # BASELINE.json configs[4] scene shape (tests/battery20230919_perf_asfctofL.py:14-88):
    # K=2, MK=[2,3], fewSamples + efficientSpSBC (T(z) compression), L=64; run with --scenes 512
    # BASELINE.json configs[3]: batch DANSE (d_batch), K=32 x 8 mics (D=39), 20 iterations, asy,
    # T = 10.01 s (non-aligned, quirk Q9); one WASN per GPU, replicas across ranks
    'D': dict(M=[8] * 32, dur=10.01, nodeUpdating='asy', batch=True, iters=20,
              desc='D: batch GEVD-DANSE r1, K=32 x 8 mics (D=39), 20 iterations, asy, 10.01 s'),
    'E_L64': dict(M=[2, 3], dur=10.0, nodeUpdating='asy', extra=dict(broadcastType='fewSamples', broadcastLength=64),
                  desc='E: GEVD-DANSE r1, K=2, MK=[2,3], fewSamples L=64 (T(z)), asy, 10 s'),
}


def _wl_params(wl):
    return _battery_params(wl['M'], wl['nodeUpdating'], **wl.get('extra', {}))


def alg_bytes_update(D, solve):
    """algorithmic HBM bytes per node x bin x frame (complex64,
    packed Hermitian): read+write the VAD-selected SCM, read y, write dhat;
    on solve frames also read the other SCM and write w."""
    b = 8 * D * (D + 1) + 8 * D + 8
    if solve:
        b += 4 * D * (D + 1) + 8 * D
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--scenes', type=int, default=31,
                    help='scenes per GPU (31 x 8 nodes x 513 bins = 1988 lane-kernel waves: ~2 full '
                         'rounds of the 1024 wave slots the update kernel can hold)')
    ap.add_argument('--workload', default='B', choices=sorted(WORKLOADS))
    ap.add_argument('--shard', default='nodes', choices=['nodes', 'scenes'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--no-traffic', action='store_true', help='skip the rocprofv3 PMC passes')
    ap.add_argument('--cpu-only', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--pmc-child', action='store_true', help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_only:
        wl = WORKLOADS[args.workload]
        dp, wp = _wl_params(wl)
        print(json.dumps(cpu_baseline(wl['M'], wl, dp, wp, args.cpu_seconds)))
        return

    import torch
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit('launch N>1 with torch.distributed.run (one process per GPU)')
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group('nccl', device_id=torch.device(f'cuda:{local}'))

    from danse_amd.engine import DanseEngine
    from danse_amd.scene import make_scene
    from danse_amd import _lib as L

    wl = WORKLOADS[args.workload]
    if wl.get('batch'):
        return bench_batch(args, wl, rank, world, local, dist)
    M = wl['M']
    K = len(M)
    dp, wp = _wl_params(wl)
    S = args.scenes
    shard = args.shard if world > 1 else 'scenes'
    if shard == 'nodes':
        if K % world != 0:
            raise SystemExit(f'K={K} not divisible by {world} ranks')
        per = K // world
        k0, k1 = rank * per, (rank + 1) * per
        Stot = S * world
        seeds = list(range(Stot))
        nodes = list(range(k0, k1))
    else:
        k0, k1 = 0, K
        Stot = S * world
        seeds = list(range(rank * S, (rank + 1) * S))
        nodes = None
    t0 = time.time()
    scenes = []
    for i, sd in enumerate(seeds):
        sc = make_scene(M, sigDur=wl['dur'], seed=1000 + sd, nodes=nodes)
        sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
        scenes.append(sc)
        if (i + 1) % 64 == 0:
            print(f'# {i + 1}/{len(seeds)} scenes generated', file=sys.stderr, flush=True)
    tScene = time.time() - t0
    eng = DanseEngine(scenes, dp, vadMinProp=wp.vadMinProportionActive, device=local, keepHistory=True,
                      nodeRange=(k0, k1))
    R, F = eng.R, eng.F
    stream = torch.cuda.current_stream()

    runner = None
    if shard == 'nodes' and world > 1:
        from danse_amd.dist import ShardedRun, ShardedEngine
        runner = ShardedRun(ShardedEngine(eng))      # per-round in-place RCCL all-gather of fused spectra

    def one_pass():
        if runner is not None:
            runner.run(reset=True)
        else:
            L.check(eng.lib.danse_engine_reset(eng.eng, eng.stream_ptr()), eng.eng)
            eng.run(graph=not args.no_graph)

    if args.pmc_child:
        # one un-graphed pass for the PMC collector (every kernel its own dispatch)
        L.check(eng.lib.danse_engine_reset(eng.eng, eng.stream_ptr()), eng.eng)
        eng.run(graph=False)
        torch.cuda.synchronize()
        eng.close()
        return
    for _ in range(args.warmup):
        one_pass()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        one_pass()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=f'cuda:{local}')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    fu_per_step = Stot * K * F * R
    value = fu_per_step * args.steps / el

    # ---- roofline of the dominant kernel: update_kernel, live HIP events
    L.check(eng.lib.danse_engine_reset(eng.eng, eng.stream_ptr()), eng.eng)
    evs = []
    for r in range(R):
        eng.bcast(r)
        if runner is not None:
            runner.exchange(r)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        eng.update(r)
        b.record(stream)
        evs.append((a, b))
    eng.finish()
    torch.cuda.synchronize()
    upd_ms = np.array([a.elapsed_time(b) for a, b in evs])
    Dk = [M[k] + K - 1 for k in range(K)]
    D = max(Dk)
    flags = eng.flags            # [R][S][4][K]
    solve = (flags[:, :, 0, :] & L.FLAG_SOLVE) != 0
    byts = []
    for r in range(R):
        b = 0
        for k in range(k0, k1):
            ns = int(solve[r, :, k].sum())
            b += F * (ns * alg_bytes_update(Dk[k], True) + (S - ns) * alg_bytes_update(Dk[k], False))
        byts.append(b)
    byts = np.array(byts, dtype=np.float64)
    avg_ms = float(upd_ms.mean())
    achieved = float(byts.mean() / (avg_ms * 1e-3) / 1e9)
    diag = eng.diagnostics()

    traffic = None
    if rank == 0 and world == 1 and not args.no_traffic:
        traffic = pmc_traffic(args, 'update_kernel')

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        import subprocess
        env = dict(os.environ, OPENBLAS_NUM_THREADS='1', MKL_NUM_THREADS='1', OMP_NUM_THREADS='1',
                   HIP_VISIBLE_DEVICES='', CUDA_VISIBLE_DEVICES='')
        env.pop('RANK', None)
        env.pop('WORLD_SIZE', None)
        cp = subprocess.run([sys.executable, str(ROOT / 'bench.py'), '--cpu-only', '--workload', args.workload,
                             '--cpu-seconds', str(args.cpu_seconds)], env=env, capture_output=True, text=True)
        try:
            cpu = json.loads(cp.stdout.strip().splitlines()[-1])
        except Exception:
            cpu = {'error': (cp.stderr or '')[-500:]}

    if rank == 0:
        line = {
            'metric': 'DANSE frame-updates/sec (nodes x bins)',
            'value': value,
            'unit': 'frame-updates/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': el / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'c64',
            'data': f'synthetic random-IR scenes (seeded), {Stot} scenes x {K} nodes x {F} bins x {R} rounds per step',
            'config': {'workload': wl['desc'], 'scenes_per_gpu': S, 'K': K, 'M': M, 'D': Dk, 'bins': F,
                       'rounds': R, 'shard': shard, 'gevd_rank': 1, 'graph': not args.no_graph},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS,
                         'traffic': (traffic or {}).get('bytes_per_launch'),
                         'traffic_detail': traffic,
                         'kernel': 'update_kernel', 'avg_launch_ms': avg_ms,
                         'alg_bytes_per_launch': float(byts.mean())},
            'cpu_baseline': cpu,
            'diag_nonpd': int(np.sum(diag)),
            'scene_gen_s': tScene,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def bench_batch(args, wl, rank, world, local, dist):
    """Batch DANSE (config D): a step is one full danse_batch run (STFT, then
    per iteration z, the MFMA Y.Y^H covariance contraction over VAD / non-VAD
    frames, every node's solve, external filters, estimates, ISTFT and MMSE
    cost) over S WASNs per GPU.  value = iterations x nodes x STFT frames x
    bins / s.  Roofline of the dominant kernel (herk_kernel) comes from the
    rocprofv3 kernel statistics of the same command, not from live
    events: the kernel is internal to danse_batch_run."""
    import torch
    from danse_amd import params as P
    from danse_amd.batch import BatchEngine
    from danse_amd.scene import make_scene
    M, K, S = wl['M'], len(wl['M']), args.scenes
    dp, wp = _battery_params(M, wl['nodeUpdating'])
    dp.simType = 'batch'
    dp.maxBatchUpdates = wl['iters']
    t0 = time.time()
    scenes = []
    for sd in range(rank * S, (rank + 1) * S):
        sc = make_scene(M, sigDur=wl['dur'], seed=2000 + sd)
        sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
        scenes.append(sc)
    tScene = time.time() - t0
    eng = BatchEngine(scenes, dp, device=local)
    for _ in range(args.warmup):
        eng.run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        eng.run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=f'cuda:{local}')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    F = eng.F
    fu_per_step = S * world * K * eng.nseg * F * eng.iters
    D = M[0] + K - 1
    herk_flops = S * K * eng.iters * 4.0 * F * D * (D + 1) * eng.nseg   # SURVEY §8d (Hermitian half)
    if rank == 0:
        line = {
            'metric': 'DANSE frame-updates/sec (nodes x bins)', 'value': fu_per_step * args.steps / el,
            'unit': 'frame-updates/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': el / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'c64',
            'data': f'synthetic random-IR scenes (seeded), {S * world} WASNs x {K} nodes x {eng.nseg} frames x {F} '
                    f'bins x {eng.iters} iterations per step',
            'config': {'workload': wl['desc'], 'wasns_per_gpu': S, 'K': K, 'M': M[0], 'D': D, 'bins': F,
                       'frames': eng.nseg, 'iterations': eng.iters, 'shard': 'replicas'},
            'roofline': None,
            'herk_alg_flops_per_step_per_gpu': herk_flops,
            'cpu_baseline': None,
            'scene_gen_s': tScene,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def pmc_traffic(args, kernel_substr):
    """HBM bytes per launch of the dominant kernel from two rocprofv3 PMC
    passes over the same workload (MI355X_MICROARCH.md, HBM section):
    FETCH_SIZE and WRITE_SIZE (KiB) in separate passes, FETCH_SIZE doubled
    (gfx950 reports half the bytes of a wide streaming read)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which('rocprofv3')
    if exe is None:
        return None
    out = {}
    tmp = tempfile.mkdtemp(prefix='danse_pmc_')
    env = dict(os.environ, TMPDIR=os.environ.get('TMPDIR', '/tmp'))
    for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
        d = os.path.join(tmp, counter)
        cmd = [exe, '--pmc', counter, '--kernel-trace', '-d', d, '-o', 'pmc', '--output-format', 'csv', '--',
               sys.executable, str(ROOT / 'bench.py'), '--pmc-child', '--workload', args.workload,
               '--scenes', str(args.scenes)]
        try:
            subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, check=True)
        except Exception as e:   # profiler unavailable or refused: report null, never fail the bench
            return {'error': f'{counter}: {type(e).__name__}'}
        files = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith('counter_collection.csv')]
        vals = [float(row['Counter_Value']) * 1024.0 for fn in files for row in csv.DictReader(open(fn))
                if row['Counter_Name'] == counter and kernel_substr in row['Kernel_Name']]
        if not vals:
            return {'error': f'{counter}: no samples'}
        out[counter] = float(np.mean(vals))
        out['dispatches'] = len(vals)
    shutil.rmtree(tmp, ignore_errors=True)
    b = 2.0 * out['FETCH_SIZE'] + out['WRITE_SIZE']
    return {'bytes_per_launch': b, 'fetch_bytes_raw': out['FETCH_SIZE'], 'write_bytes': out['WRITE_SIZE'],
            'dispatches': out['dispatches'], 'method': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, '
            'FETCH_SIZE x2 (gfx950)'}


def ctypes_void(p):
    import ctypes
    return ctypes.c_void_p(p)


def cpu_baseline(M, wl, dp, wp, seconds):
    """The float64 oracle (oracle/danse_ref_cpu.py, same NumPy/SciPy calls as
    the reference) on one scene of the workload, single process, default BLAS
    threads; FU/s over the steady-state rounds (every node past the gate)."""
    from danse_amd.scene import make_scene
    from oracle import danse_ref_cpu as O
    sc = make_scene(M, sigDur=wl['dur'], seed=1000)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    K, F = len(M), dp.DFTsize // 2 + 1
    # gate round from the counters (the oracle reproduces it exactly)
    D = max(M) + K - 1
    starts = []
    for nd in sc.wasn:
        v = nd.vadPerFrame
        ny = np.cumsum(v)
        nn = np.arange(1, len(v) + 1) - ny
        starts.append(int(np.argmax((ny > D) & (nn > D))))
    r0 = max(starts) + 1
    # estimate per-round cost from a short probe, then size the window to ~seconds
    probe = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive, maxRounds=r0 + 2)
    t = time.perf_counter()
    probe.run()
    rt = probe.roundTimes
    per_round = (rt[-1][1] - [x for x in rt if x[0] >= r0][0][1]) / 2.0
    nwin = int(max(4, min(300 - r0, seconds / max(per_round, 1e-3))))
    ov = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive, maxRounds=r0 + nwin)
    ov.run()
    rt = ov.roundTimes
    tA = [x for x in rt if x[0] >= r0][0][1]
    tB = rt[-1][1]
    fu = K * F * nwin
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count()
    return {'value': fu / (tB - tA), 'unit': 'frame-updates/s', 'cores': 1, 'kind': 'port',
            'sample': f'oracle float64 (numpy/scipy eigh per bin), one process, BLAS/OMP threads = 1, scene seed '
                      f'1000, rounds {r0}..{r0 + nwin} (all {K} nodes past the gate), {tB - tA:.1f} s; '
                      f'host affinity {cores} cpus'}


if __name__ == '__main__':
    main()
