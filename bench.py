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

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md, chip-level parameters
FP32_VALU_PEAK_TFS = 157.3    # ibid., peak FP32 (vector)
FP32_MFMA_PEAK_TFS = 157.3    # ibid., peak FP32 (matrix, f32-input MFMA: the vector rate on gfx950)
OP_KEEP, OP_SET, OP_AVG = 0, 1, 2   # include/danse_mi355x_defs.h DANSE_OP_* (danse_amd._lib OP_*)


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
    'B': dict(M=[4] * 8, dur=10.0, nodeUpdating='asy', scenes=31,
              desc='B: GEVD-DANSE r1, K=8 x 4 mics, N=1024, asy, 10 s'),
    # north_star headline shape: online, 32 nodes x 8 mics (D = 39), 513 bins, one WASN per GPU
    'N2': dict(M=[8] * 32, dur=10.0, nodeUpdating='asy', scenes=1,
               desc='N2: online GEVD-DANSE r1, K=32 x 8 mics (D=39), N=1024, asy, 10 s, single WASN'),
    # BASELINE.json configs[2]: online, K = 16 x 4 (D = 19), SROs up to 200 ppm with
    # data-driven SRO estimation (CohDrift, closed loop, least squares) and
    # phase compensation; 8 WASNs per GPU
    'C': dict(M=[4] * 16, dur=10.0, nodeUpdating='asy', scenes=8, sros=[float(x) for x in np.linspace(0, 200, 16)],
              extra=dict(compensateSROs=True, includeFSDflags=True, estimateSROs='CohDrift', cohdrift_ls=True),
              desc='C: GEVD-DANSE r1, K=16 x 4 mics (D=19), SROs 0..200 ppm, CohDrift estimation + compensation, asy, 10 s'),
    # BASELINE.json configs[2] as named: DXCP-PhaT SRO estimation (the
    # device estimators per (receiver, sender) pair on the received z
    # streams, danse_cfg.dxcp) + compensation, K = 16 x 4, SROs 0..200 ppm
    'C_dxcp': dict(M=[4] * 16, dur=10.0, nodeUpdating='asy', scenes=8, sros=[float(x) for x in np.linspace(0, 200, 16)],
                   extra=dict(compensateSROs=True, includeFSDflags=True, estimateSROs='DXCPPhaT'),
                   desc='C: GEVD-DANSE r1, K=16 x 4 mics (D=19), SROs 0..200 ppm, DXCP-PhaT estimation + '
                        'compensation, asy, 10 s'),
    'B_seq': dict(M=[4] * 8, dur=10.0, nodeUpdating='seq', scenes=31, desc='B (seq): GEVD-DANSE r1, K=8 x 4 mics, seq, 10 s'),
    'small': dict(M=[2] * 4, dur=3.0, nodeUpdating='asy', desc='small smoke workload K=4 x 2, 3 s'),
    # BASELINE.json configs[4] scene shape (tests/battery20230919_perf_asfctofL.py:14-88):
    # K=2, MK=[2,3], fewSamples + efficientSpSBC (T(z) compression), L=64; run with --scenes 512
    # BASELINE.json configs[3]: batch DANSE (d_batch), K=32 x 8 mics (D=39), 20 iterations, asy,
    # T = 10.01 s (non-aligned, quirk Q9); one WASN per GPU, replicas across ranks
    'D': dict(M=[8] * 32, dur=10.01, nodeUpdating='asy', batch=True, iters=20,
              desc='D: batch GEVD-DANSE r1, K=32 x 8 mics (D=39), 20 iterations, asy, 10.01 s'),
    'E_L64': dict(M=[2, 3], dur=10.0, nodeUpdating='asy', extra=dict(broadcastType='fewSamples', broadcastLength=64),
                  desc='E: GEVD-DANSE r1, K=2, MK=[2,3], fewSamples L=64 (T(z)), asy, 10 s'),
    # the battery's SRO setting (config_files/sandbox_config_battery20230919.yaml:24-25): node 2 at
    # 200 ppm, Oracle estimates, compensation with full-sample-drift flags (no centralised family:
    # centralised estimates under SRO clocks are not on the device path)
    'E_L64_sro200': dict(M=[2, 3], dur=10.0, nodeUpdating='asy', sros=[0.0, 200.0],
                         extra=dict(broadcastType='fewSamples', broadcastLength=64, compensateSROs=True,
                                    includeFSDflags=True),
                         desc='E: GEVD-DANSE r1, K=2, MK=[2,3], fewSamples L=64, SROs [0, 200] ppm + compensation, '
                              'asy, 10 s'),
    # the battery itself (tests/battery20230919_perf_asfctofL.py:60-104): SROs [0, 200] ppm, Oracle
    # estimates, sandbox_config.yaml families on (local, centralised, SSBC: SSBC with compensation
    # raises in the reference, d_classes.py:2042-2044, so the comp variants run local + centralised);
    # --L sets broadcastLength (every L in divisors(512): scheduler.compile_rounds_fs step lists)
    'E_noComp': dict(M=[2, 3], dur=10.0, nodeUpdating='asy', sros=[0.0, 200.0],
                     extra=dict(broadcastType='fewSamples', broadcastLength=64, compensateSROs=False,
                                computeLocal=True, computeCentralised=True, computeSingleSensorBroadcast=True),
                     desc='E battery noComp: K=2, MK=[2,3], fewSamples L, SROs [0, 200] ppm, no compensation, '
                          'DANSE + local + centralised + SSBC, asy, 10 s'),
    'E_compNoFlags': dict(M=[2, 3], dur=10.0, nodeUpdating='asy', sros=[0.0, 200.0],
                          extra=dict(broadcastType='fewSamples', broadcastLength=64, compensateSROs=True,
                                     includeFSDflags=False, computeLocal=True, computeCentralised=True),
                          desc='E battery compNoFlags: K=2, MK=[2,3], fewSamples L, SROs [0, 200] ppm, Oracle '
                               'compensation without flags, DANSE + local + centralised, asy, 10 s'),
    'E_comp': dict(M=[2, 3], dur=10.0, nodeUpdating='asy', sros=[0.0, 200.0],
                   extra=dict(broadcastType='fewSamples', broadcastLength=64, compensateSROs=True,
                              includeFSDflags=True, computeLocal=True, computeCentralised=True),
                   desc='E battery comp: K=2, MK=[2,3], fewSamples L, SROs [0, 200] ppm, Oracle compensation with '
                        'flags, DANSE + local + centralised, asy, 10 s'),
}


for _n, _w in WORKLOADS.items():
    _w['name'] = _n

_CHILD_ARGS = []   # workload overrides forwarded to the CPU-baseline and PMC child processes


def _wl_params(wl):
    extra = dict(wl.get('extra', {}))
    if extra.pop('cohdrift_ls', False):
        from danse_amd import params as P
        extra['cohDrift'] = P.CohDriftParameters(estimationMethod='ls')
    return _battery_params(wl['M'], wl['nodeUpdating'], **extra)


def update_kernel_name(Dmax, gevd=True):
    """The update kernel a filter dimension runs on (danse_amd/csrc/update_class.hip)."""
    if Dmax <= 12:
        return 'update_kernel_lane'
    return 'update_kernel_2d' if (gevd and Dmax <= 48) else 'update_kernel_big'


def update_kernel_mix(Dmax, gevd=True):
    """The kernels one solve round's update launches run at filter size Dmax
    (danse_engine.hip launch_update): the lean cached-C solves of the 8 x 8
    grid classes (DMAX 24-48, rank 1) sit beside the full kernel."""
    k = update_kernel_name(Dmax, gevd)
    if k == 'update_kernel_2d' and Dmax > 20:
        return 'update_kernel_2d + update_kernel_2dc<VAD> + update_kernel_2dc<noise> + fallback_kernel_2d'
    return k


def alg_bytes_update(D, opY, opN, solve):
    """Algorithmic HBM bytes of one node x bin x frame of update_kernel,
    SURVEY §8d (complex64, packed Hermitian: one SCM one way = 4 D(D+1) B):
    read y (8 D), write dhat (8); read + write the SCM this frame's VAD
    updates (DANSE_OP_AVG: 8 D(D+1)), or write it only when the first frame
    sets it (DANSE_OP_SET: 4 D(D+1)); on solve frames also read the SCM left
    alone (4 D(D+1)) and write w (8 D).  Arrays of per-frame op codes / solve
    flags in, bytes out."""
    opY, opN, solve = np.asarray(opY), np.asarray(opN), np.asarray(solve)
    t = D * (D + 1)
    one = 4.0 * t

    def scm(op):
        return np.where(op == OP_AVG, 2.0 * one, np.where(op == OP_SET, one, np.where(solve, one, 0.0)))
    return 8.0 * D + 8.0 + scm(opY) + scm(opN) + np.where(solve, 8.0 * D, 0.0)


def storage_bytes_update(D, opY, opN, solve):
    """The same frame in the engine's storage: Ryy packed
    complex64 (4 D(D+1) B one way), Rnn packed complex128 (8 D(D+1) B), w
    read from the previous slot and written to the next on frames without a
    solve (16 D) or written only (8 D); the GEVD factor caches not counted."""
    opY, opN, solve = np.asarray(opY), np.asarray(opN), np.asarray(solve)
    t = D * (D + 1)

    def scm(op, one):
        return np.where(op == OP_AVG, 2.0 * one, np.where(op == OP_SET, one, np.where(solve, one, 0.0)))
    return (8.0 * D + 8.0 + scm(opY, 4.0 * t) + scm(opN, 8.0 * t) + np.where(solve, 8.0 * D, 16.0 * D))


def alg_flops_update(D, opY, opN, solve):
    """Algorithmic flops of one node x bin x frame of update_kernel (SURVEY
    §8d): SCM recursion 5 D(D+1); on solve frames the rank-1 GEVD filter as
    LAPACK counts it, zpotrf + zhegst + zhetrd = (32/3) D^3, plus the
    eigenvector back-transform and x = L^-H v (12 D^2); dhat 8 D."""
    opY, opN, solve = np.asarray(opY), np.asarray(opN), np.asarray(solve)
    f = 8.0 * D + np.where((opY != 0) | (opN != 0), 5.0 * D * (D + 1), 0.0)
    return f + np.where(solve, 32.0 / 3.0 * D ** 3 + 12.0 * D * D, 0.0)


# D above which the fused update + GEVD solve crosses the fp32-vector ridge
# (157.3 TF / 8 TB/s ~ 20 flop/B; SURVEY §8d "Which roofline").
VALU_RIDGE_D = 22


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--scenes', type=int, default=None,
                    help='scenes per GPU (B default 31: 31 x 8 nodes x 513 bins = 1988 lane-kernel waves, '
                         '~2 full rounds of the 1024 wave slots the update kernel can hold; N2 default 1)')
    ap.add_argument('--workload', default='B', choices=sorted(WORKLOADS))
    ap.add_argument('--shard', default='nodes', choices=['nodes', 'scenes'])
    ap.add_argument('--batch-shard', default='replicas', choices=['replicas', 'nodes'],
                    help='config D on N>1 GPUs: independent WASNs per GPU (weak scaling) or every GPU owning a '
                         'node block of the same WASNs, external filters all-gathered per iteration (strong)')
    ap.add_argument('--L', type=int, default=None, help='broadcastLength override (fewSamples workloads)')
    ap.add_argument('--scene-gen', default='auto', choices=['auto', 'host', 'device'],
                    help='synthetic scenes from the host generator (danse_amd.scene.make_scene) or the device one '
                         '(csrc/scene.hip, with SRO resampling); auto: device from 64 scenes per GPU on')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--resident', action='store_true', help='online workloads: the resident engine (one persistent launch)')
    ap.add_argument('--small-grid', action='store_true',
                    help='online workloads: GEVD of D <= 12 on the 4 x 4 lane-grid class instead of one bin per lane')
    ap.add_argument('--no-traffic', action='store_true', help='skip the rocprofv3 PMC passes')
    ap.add_argument('--no-extra', action='store_true',
                    help='N=1, workload B: skip the extra single-WASN lines (B at S=1, N2 K=32x8 at S=1)')
    ap.add_argument('--cpu-only', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--rounds', type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument('--cpu-seed', type=int, default=1000, help=argparse.SUPPRESS)
    ap.add_argument('--pmc-child', action='store_true', help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.L is not None:
        w = WORKLOADS[args.workload]
        if w.get('extra', {}).get('broadcastType') != 'fewSamples':
            raise SystemExit('--L applies to the fewSamples workloads')
        w['extra'] = dict(w['extra'], broadcastLength=int(args.L))
        w['desc'] = w['desc'].replace('fewSamples L=64', f'fewSamples L={args.L}').replace('fewSamples L,', f'fewSamples L={args.L},')
    _CHILD_ARGS.extend(['--L', str(args.L)] if args.L is not None else [])
    _CHILD_ARGS.extend(['--small-grid'] if args.small_grid else [])
    if args.cpu_only:
        wl = WORKLOADS[args.workload]
        if wl.get('batch'):
            dp, wp = _battery_params(wl['M'], wl['nodeUpdating'])
            dp.simType = 'batch'
            dp.maxBatchUpdates = wl['iters']
            print(json.dumps(cpu_baseline_batch(wl['M'], wl, dp, wp, args.cpu_seconds)))
            return
        dp, wp = _wl_params(wl)
        print(json.dumps(cpu_baseline(wl['M'], wl, dp, wp, args.cpu_seconds, args.rounds, seed=args.cpu_seed)))
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

    wl = WORKLOADS[args.workload]
    S = args.scenes if args.scenes is not None else wl.get('scenes', 1)
    if wl.get('batch'):
        return bench_batch(args, wl, S, rank, world, local, dist)
    if args.pmc_child:
        run_online(args, wl, S, rank, world, local, dist, pmc_child=True, small_grid=args.small_grid)
        return
    res = run_online(args, wl, S, rank, world, local, dist, resident=args.resident, small_grid=args.small_grid)
    _progress(f'{args.workload}: {res["value"] / 1e6:.1f} M FU/s')
    extra = {}
    if world == 1 and args.workload == 'B' and not args.no_extra:
        # single-WASN lines: config B at S=1 and the
        # north_star headline shape N2 (online K=32 x 8, D=39) at S=1
        extra['B_S1'] = run_online(args, wl, 1, rank, world, local, dist, traffic=False)
        _progress(f'B_S1: {extra["B_S1"]["value"] / 1e6:.1f} M FU/s')
        # the latency layout for one WASN: D = 11 on the 4 x 4 lane-grid solver
        extra['B_S1_grid'] = run_online(args, wl, 1, rank, world, local, dist, traffic=False, small_grid=True)
        _progress(f'B_S1_grid: {extra["B_S1_grid"]["value"] / 1e6:.1f} M FU/s')
        # N1: the whole run in one persistent launch, SCMs resident in registers
        extra['B_S1_resident'] = run_online(args, wl, 1, rank, world, local, dist, traffic=False, resident=True)
        _progress(f'B_S1_resident: {extra["B_S1_resident"]["value"] / 1e6:.1f} M FU/s')
        extra['N2'] = run_online(args, WORKLOADS['N2'], 1, rank, world, local, dist)
        _progress(f'N2: {extra["N2"]["value"] / 1e6:.1f} M FU/s')
        # the other BASELINE.json configs, each on its own shape: C as named
        # (DXCP-PhaT estimation + compensation, K = 16 x 4, SROs 0..200 ppm),
        # D (batch K = 32 x 8, 20 iterations) and E at the battery's SRO
        # setting (K = 2, MK = [2, 3], fewSamples L = 64, 512 scenes)
        extra['C_dxcp'] = run_online(args, WORKLOADS['C_dxcp'], WORKLOADS['C_dxcp']['scenes'], rank, world, local,
                                     dist)
        _progress(f'C_dxcp: {extra["C_dxcp"]["value"] / 1e6:.1f} M FU/s')
        extra['D'] = run_batch(args, WORKLOADS['D'], 1, rank, world, local, dist)
        _progress(f'D: {extra["D"]["value"] / 1e6:.1f} M FU/s')
        extra['E_L64_sro200'] = run_online(args, WORKLOADS['E_L64_sro200'], 512, rank, world, local, dist,
                                           traffic=False)
        _progress(f'E_L64_sro200: {extra["E_L64_sro200"]["value"] / 1e6:.1f} M FU/s')
        # the battery's cell as the battery configures it (local and
        # centralised families on, Oracle compensation with flags; FU counts
        # the DANSE family, the other families are extra solves)
        extra['E_comp'] = run_online(args, WORKLOADS['E_comp'], 512, rank, world, local, dist, traffic=False)
        _progress(f'E_comp: {extra["E_comp"]["value"] / 1e6:.1f} M FU/s')
    cpu = {}
    if rank == 0 and not args.no_cpu_baseline:
        _progress(f'CPU leg {args.workload}')
        cpu[args.workload] = cpu_child(args.workload, args.cpu_seconds, res['rounds'])
        for key in ('N2', 'C_dxcp', 'D', 'E_L64_sro200', 'E_comp'):
            if key in extra:
                _progress(f'CPU leg {key}')
                cpu[key] = cpu_child(key, args.cpu_seconds, extra[key].get('rounds'))
        for key in ('E_L64_sro200', 'E_comp'):
            # for E also a P-process scene-parallel CPU leg (a
            # shorter budget per process: they run at once)
            if key in extra and cpu.get(key) and 'value' in cpu[key]:
                _progress(f'CPU leg {key}, scene-parallel')
                cpu[key]['scene_parallel'] = cpu_parallel(key, min(args.cpu_seconds, 8.0), extra[key].get('rounds'))
    if rank == 0:
        line = {
            'metric': 'DANSE frame-updates/sec (nodes x bins)',
            'value': res['value'],
            'unit': 'frame-updates/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': res['ms_per_step'],
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'c64',
            'data': res['data'],
            'config': res['config'],
            'roofline': res['roofline'],
            'cpu_baseline': cpu.get(args.workload),
            'diag_nonpd': res['diag_nonpd'],
            'scene_gen_s': res['scene_gen_s'],
        }
        if extra:
            line['extra_lines'] = {}
            for key, r in extra.items():
                c = cpu.get(key)
                if key in ('B_S1', 'B_S1_grid', 'B_S1_resident'):
                    c = cpu.get('B')
                line['extra_lines'][key] = {
                    'value': r['value'], 'unit': 'frame-updates/s', 'ms_per_step': r['ms_per_step'],
                    'data': r['data'], 'config': r['config'], 'roofline': r['roofline'],
                    'cpu_baseline': c,
                    'gpu_over_cpu': (r['value'] / c['value']) if c and c.get('value') else None,
                }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _progress(msg):
    """A progress line on stderr (long default runs stay visibly alive)."""
    print(f'# [{time.strftime("%H:%M:%S")}] {msg}', file=sys.stderr, flush=True)


def cpu_child(workload, seconds, rounds):
    """The CPU leg in a child process without the GPU (BLAS at its default
    thread count)."""
    import subprocess
    env = dict(os.environ, HIP_VISIBLE_DEVICES='', CUDA_VISIBLE_DEVICES='', ROCR_VISIBLE_DEVICES='')
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK'):
        env.pop(k, None)
    cmd = [sys.executable, str(ROOT / 'bench.py'), '--cpu-only', '--workload', workload, '--cpu-seconds', str(seconds),
           *_CHILD_ARGS]
    if rounds is not None:
        cmd += ['--rounds', str(rounds)]
    cp = subprocess.run(cmd,
                        env=env, capture_output=True, text=True)
    try:
        return json.loads(cp.stdout.strip().splitlines()[-1])
    except Exception:
        return {'error': (cp.stderr or '')[-500:]}


def cpu_parallel(workload, seconds, rounds):
    """The scene-parallel CPU leg: P = the host's
    CPU share (affinity, capped by the thread-count env the box sets) single-
    threaded oracle processes, each on its own scene seed, run at once; the
    aggregate is the sum of their frame-update rates over the common wall."""
    import subprocess
    cores, threads, env0 = _threads()
    P = max(1, threads)
    env = dict(os.environ, HIP_VISIBLE_DEVICES='', CUDA_VISIBLE_DEVICES='', ROCR_VISIBLE_DEVICES='',
               OMP_NUM_THREADS='1', OPENBLAS_NUM_THREADS='1', MKL_NUM_THREADS='1')
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK'):
        env.pop(k, None)
    t0 = time.perf_counter()
    procs = []
    for i in range(P):
        cmd = [sys.executable, str(ROOT / 'bench.py'), '--cpu-only', '--workload', workload, '--cpu-seconds',
               str(seconds), '--cpu-seed', str(1000 + i), *_CHILD_ARGS]
        if rounds is not None:
            cmd += ['--rounds', str(rounds)]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    vals, errs = [], []
    for pr in procs:
        o, e = pr.communicate()
        try:
            vals.append(json.loads(o.strip().splitlines()[-1])['value'])
        except Exception:
            errs.append((e or '')[-200:])
    wall = time.perf_counter() - t0
    if not vals:
        return {'error': errs[:1]}
    return {'value': float(np.sum(vals)), 'unit': 'frame-updates/s', 'cores': P, 'processes': len(vals),
            'kind': 'port', 'per_process_median': float(np.median(vals)), 'wall_s': wall,
            'sample': f'{len(vals)} concurrent single-threaded float64 oracle processes (scene seeds 1000..'
                      f'{1000 + P - 1}), each timed as the one-process leg; value = the sum of their rates; host '
                      f'affinity {cores} cpus, thread env {env0 or "unset"}'}


def run_online(args, wl, S, rank, world, local, dist, traffic=True, pmc_child=False, small_grid=False, resident=False):
    """One online-engine measurement: S scenes per GPU of workload wl.  A
    step is one full pass of the engine (state reset + every round: WOLA
    analysis, compression, z synthesis, SCM update, GEVD filter update,
    external filters, estimate synthesis) with the inputs resident in HBM."""
    import torch
    from danse_amd.engine import DanseEngine
    from danse_amd.scene import make_scene
    from danse_amd import _lib as L
    M = wl['M']
    K = len(M)
    dp, wp = _wl_params(wl)
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
    gen = args.scene_gen if args.scene_gen != 'auto' else ('device' if len(seeds) >= 64 else 'host')
    yDev = None
    if gen == 'device':
        from danse_amd.scene import make_scenes_device
        scenes, dev = make_scenes_device(M, len(seeds), sigDur=wl['dur'], seed=1000 + seeds[0],
                                         SROperNode=wl.get('sros'), device=local)
        yDev = dev['data']
        for sc in scenes:
            sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
        torch.cuda.synchronize()
    else:
        for i, sd in enumerate(seeds):
            sc = make_scene(M, sigDur=wl['dur'], seed=1000 + sd, nodes=nodes, SROperNode=wl.get('sros'))
            sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
            scenes.append(sc)
            if (i + 1) % 64 == 0:
                print(f'# {i + 1}/{len(seeds)} scenes generated', file=sys.stderr, flush=True)
    tScene = time.time() - t0
    eng = DanseEngine(scenes, dp, vadMinProp=wp.vadMinProportionActive, device=local, keepHistory=True,
                      nodeRange=(k0, k1), yDevice=yDev, smallDGrid=small_grid, resident=resident)
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
            eng.run(graph=not args.no_graph)     # (every run starts with the state reset)

    if pmc_child:
        # one un-graphed pass for the PMC collector (every kernel its own dispatch)
        L.check(eng.lib.danse_engine_reset(eng.eng, eng.stream_ptr()), eng.eng)
        eng.run(graph=False)
        torch.cuda.synchronize()
        eng.close()
        return None
    # with the node-sharded runner the barriers and the max over ranks go
    # over its gloo control group: an RCCL collective outside the captured
    # rounds would corrupt the later graph replays (danse_amd/dist.py)
    ctl = runner.ctl if runner is not None else None
    for _ in range(args.warmup):
        one_pass()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier(group=ctl)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        one_pass()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier(group=ctl)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device='cpu' if ctl is not None else f'cuda:{local}')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=ctl)
        el = float(tt.item())
    fu_per_step = Stot * K * F * R
    value = fu_per_step * args.steps / el

    # ---- roofline of the dominant kernel (update_kernel): live HIP events on
    # the engine's stream around each round's update launch
    L.check(eng.lib.danse_engine_reset(eng.eng, eng.stream_ptr()), eng.eng)
    evs = []
    if resident:
        # one persistent launch per run: the "launch" is the whole run
        # (analyses, round loop, gate checks, synthesis) on the engine stream
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        eng.run()
        b.record(stream)
        evs.append((a, b))
    for r in range(R if not resident else 0):
        eng.bcast(r)
        if runner is not None:
            runner.exchange(r)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        eng.update(r)
        b.record(stream)
        evs.append((a, b))
    if not resident:
        eng.finish()
    torch.cuda.synchronize()
    upd_ms = np.array([a.elapsed_time(b) for a, b in evs])
    Dk = [M[k] + K - 1 for k in range(K)]
    fl = eng.flags[:, :, 0, k0:k1].astype(np.int64)        # [R][S][local nodes]
    opY, opN = fl & 3, (fl >> 2) & 3
    solve = ((fl & L.FLAG_SOLVE) != 0) & ((fl & L.FLAG_PREGIVEN) == 0)
    Dl = np.array(Dk[k0:k1], dtype=np.float64)[None, None, :]
    byts = F * alg_bytes_update(Dl, opY, opN, solve).sum(axis=(1, 2))       # per launch (round)
    sbyts = F * storage_bytes_update(Dl, opY, opN, solve).sum(axis=(1, 2))
    flops = F * alg_flops_update(Dl, opY, opN, solve).sum(axis=(1, 2))
    # the dominant kernel: the update launches of the rounds with a solving
    # item (the solver instantiation); the recursion-only rounds run the
    # recursion-only variants (UpdateArgs.noSolve) and are reported apart
    solveRound = solve.any(axis=(1, 2))
    if resident:
        # per launch = every round of the run
        byts, sbyts, flops = np.array([byts.sum()]), np.array([sbyts.sum()]), np.array([flops.sum()])
        dom = np.array([True])
    else:
        dom = solveRound if solveRound.any() else np.ones_like(solveRound)
    avg_ms = float(upd_ms[dom].mean())
    gbs = float(byts[dom].mean() / (avg_ms * 1e-3) / 1e9)
    sgbs = float(sbyts[dom].mean() / (avg_ms * 1e-3) / 1e9)
    tfs = float(flops[dom].mean() / (avg_ms * 1e-3) / 1e12)
    rec = None
    if not resident and (~dom).any():
        rms = float(upd_ms[~dom].mean())
        rec = {'rounds': int((~dom).sum()), 'avg_launch_ms': rms,
               'alg_bytes_per_launch': float(byts[~dom].mean()),
               'hbm_GBs': float(byts[~dom].mean() / (rms * 1e-3) / 1e9)}
    diag = eng.diagnostics()
    lz = eng.lanczos_stats()
    eng.close()

    tr = None
    if traffic and rank == 0 and world == 1 and not args.no_traffic:
        # (the round groups need one broadcast dispatch per round: wholeChunk)
        fs = wl.get('extra', {}).get('broadcastType') == 'fewSamples'
        if resident:
            tr = pmc_traffic(wl, S, 'resident_kernel')
        elif fs:
            tr = pmc_traffic(wl, S, 'update_kernel', dom)
        else:
            tr = pmc_traffic(wl, S, None, dom)
    valu = max(Dk) > VALU_RIDGE_D
    roof = {'bound': 'valu' if valu else 'hbm',
            'achieved': tfs if valu else gbs,
            'peak': FP32_VALU_PEAK_TFS if valu else HBM_PEAK_GBS,
            'unit': 'TFLOP/s' if valu else 'GB/s',
            'frac': tfs / FP32_VALU_PEAK_TFS if valu else gbs / HBM_PEAK_GBS,
            'traffic': (tr or {}).get('bytes_per_launch'),
            'traffic_detail': tr,
            'kernel': ('resident_kernel (one persistent launch per run; achieved = all rounds\' algorithmic bytes '
                       '/ the run)' if resident else
                       'the update launches of the solve rounds (' +
                       ('update_kernel_2d (4 x 4 grid)' if small_grid and max(Dk) <= 12
                        else update_kernel_mix(max(Dk), gevd=bool(wl.get('gevd', True))))
                       + f'), {int(dom.sum())} of {R} rounds; the measured dispatch mix in traffic_detail.kernel_mix'),
            'avg_launch_ms': avg_ms,
            'alg_bytes_per_launch': float(byts[dom].mean()), 'alg_flops_per_launch': float(flops[dom].mean()),
            'bytes_model': 'SURVEY §8d: complex64 packed Hermitian SCMs (achieved); storage_* = the engine\'s '
                           'storage (Ryy c64, Rnn c128, w ring), factor caches not counted',
            'storage_bytes_per_launch': float(sbyts[dom].mean()), 'storage_GBs': sgbs,
            'hbm_GBs': gbs, 'hbm_frac': gbs / HBM_PEAK_GBS, 'valu_TFs': tfs, 'valu_frac': tfs / FP32_VALU_PEAK_TFS,
            'recursion_rounds': rec}
    if lz.any():
        roof['lanczos'] = {'accepted': int(lz[:, 0].sum()), 'sent_back': int(lz[:, 1].sum()),
                           'max_sent_back_per_launch': int(lz[:, 1].max())}
    return {
        'value': value, 'ms_per_step': el / args.steps * 1e3, 'rounds': R,
        'data': f'synthetic random-IR scenes (seeded, {gen} generator{", SRO-resampled" if gen == "device" and wl.get("sros") else ""}), '
                f'{Stot} scenes x {K} nodes x {F} bins x {R} rounds per step',
        'config': {'workload': wl['desc'], 'scenes_per_gpu': S, 'K': K, 'M': M if len(set(M)) > 1 else M[0],
                   'D': Dk if len(set(Dk)) > 1 else Dk[0], 'bins': F, 'rounds': R, 'shard': shard,
                   'gevd_rank': 1, 'graph': not args.no_graph, 'resident': resident},
        'roofline': roof, 'diag_nonpd': int(np.sum(diag)), 'scene_gen_s': tScene,
    }


def bench_batch(args, wl, S, rank, world, local, dist):
    """The batch workload (config D) as the bench line: run_batch + the CPU
    leg of rank 0."""
    res = run_batch(args, wl, S, rank, world, local, dist)
    if res is None:   # (--pmc-child)
        return
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_child(args.workload, args.cpu_seconds, None)
    if rank == 0:
        line = {
            'metric': 'DANSE frame-updates/sec (nodes x bins)', 'value': res['value'],
            'unit': 'frame-updates/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': res['ms_per_step'], 'higher_is_better': True,
            'scaling': res['scaling'], 'vs_baseline': None, 'dtype': 'c64',
            'data': res['data'], 'config': res['config'], 'roofline': res['roofline'],
            'cpu_baseline': cpu, 'scene_gen_s': res['scene_gen_s'],
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_batch(args, wl, S, rank, world, local, dist):
    """Batch DANSE (config D): a step is one full danse_batch run (STFT, then
    per iteration z, the MFMA Y.Y^H covariance contraction over VAD / non-VAD
    frames, every node's solve, external filters, estimates, ISTFT and MMSE
    cost) over S WASNs per GPU.  value = iterations x nodes x STFT frames x
    bins / s.  Roofline of the dominant kernel (herk_kernel) from live HIP
    events at the run's phase boundaries (danse_batch_set_timing), in a
    separate pass after the timed steps."""
    import torch
    from danse_amd.batch import BatchEngine
    from danse_amd.scene import make_scene
    M, K = wl['M'], len(wl['M'])
    dp, wp = _battery_params(M, wl['nodeUpdating'])
    dp.simType = 'batch'
    dp.maxBatchUpdates = wl['iters']
    t0 = time.time()
    byNodes = dist is not None and world > 1 and args.batch_shard == 'nodes'
    scenes = []
    for sd in (range(S) if byNodes else range(rank * S, (rank + 1) * S)):
        sc = make_scene(M, sigDur=wl['dur'], seed=2000 + sd)
        sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
        scenes.append(sc)
    tScene = time.time() - t0
    if byNodes:
        from danse_amd.batch import node_ranges, run_node_sharded, allgather_exchange
        rngs, blk = node_ranges(K, world)
        eng = BatchEngine(scenes, dp, device=local, nodeRange=rngs[rank])
        ex = allgather_exchange(dist, world)
        step = lambda: run_node_sharded(eng, ex, blk)   # noqa: E731
    else:
        eng = BatchEngine(scenes, dp, device=local)
        step = eng.run
    if args.pmc_child:
        # one run for the PMC collector (every kernel its own dispatch)
        step()
        torch.cuda.synchronize()
        return None
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
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
    fu_per_step = S * (1 if byNodes else world) * K * eng.nseg * F * eng.iters
    D = M[0] + K - 1
    eng.set_timing(True)
    step()
    torch.cuda.synchronize()
    ph = eng.phase_ms()
    eng.set_timing(False)
    nOwn = eng.k1 - eng.k0
    it = eng.iters
    # HERK (Hermitian half) 4 F D (D + 1) T flops per node per iteration
    herk_flops = S * nOwn * 4.0 * F * D * (D + 1) * eng.nseg
    herk_tfs = herk_flops / (ph['herk'] / it * 1e-3) / 1e12
    # GEVD solve (rank 1), LAPACK count as in the online roofline: (32/3) D^3 + 12 D^2 per bin
    solve_flops = S * nOwn * F * (32.0 / 3.0 * D ** 3 + 12.0 * D * D)
    solve_tfs = solve_flops / (ph['solve'] / it * 1e-3) / 1e12
    # dhat: read Y (the node's M channels) + Z (K - 1 fused), write dhat: 8 (D + 1) bytes per (node, bin, frame)
    dhat_bytes = S * nOwn * F * (eng.nseg - 1) * 8.0 * (D + 1)
    dhat_gbs = dhat_bytes / (ph['dhat'] / it * 1e-3) / 1e9
    roof = {'bound': 'mfma', 'kernel': 'herk_kernel (Y.Y^H, f32 MFMA 16x16x4)', 'achieved': herk_tfs,
            'peak': FP32_MFMA_PEAK_TFS, 'unit': 'TFLOP/s', 'frac': herk_tfs / FP32_MFMA_PEAK_TFS, 'traffic': None,
            'avg_launch_ms': ph['herk'] / it, 'alg_flops_per_launch': herk_flops,
            'phase_ms_per_iteration': {k: v / it for k, v in ph.items()},
            'solve': {'kernel': 'filter_update_kernel_2d (GEVD rank 1)', 'bound': 'valu', 'achieved': solve_tfs,
                      'peak': FP32_VALU_PEAK_TFS, 'unit': 'TFLOP/s', 'frac': solve_tfs / FP32_VALU_PEAK_TFS},
            'dhat': {'kernel': 'batch_dhat_kernel', 'bound': 'hbm', 'achieved': dhat_gbs, 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': dhat_gbs / HBM_PEAK_GBS}}
    eng.close()
    return {
        'value': fu_per_step * args.steps / el, 'ms_per_step': el / args.steps * 1e3,
        'scaling': 'strong' if byNodes else 'weak',
        'data': f'synthetic random-IR scenes (seeded), {S * (1 if byNodes else world)} WASNs x {K} nodes x {eng.nseg} '
                f'frames x {F} bins x {eng.iters} iterations per step',
        'config': {'workload': wl['desc'], 'wasns_per_gpu': S, 'K': K, 'M': M[0], 'D': D, 'bins': F,
                   'frames': eng.nseg, 'iterations': eng.iters, 'shard': 'nodes' if byNodes else 'replicas'},
        'roofline': roof, 'scene_gen_s': tScene,
    }


def cpu_baseline_batch(M, wl, dp, wp, seconds):
    """The float64 CPU oracle of batch DANSE (oracle/danse_ref_cpu.py
    BatchDANSE: the reference's d_batch / d_core.danse_batch algorithm,
    per-bin scipy.linalg.eigh), one process, default BLAS threads, timed on
    this host on a bounded sample: the first iteration's per-node work
    (y-tilde, both batch SCMs, GEVD solve, external filters, estimate + ISTFT,
    MMSE cost) for as many nodes as fit the time budget, projected over
    K nodes x the workload's iterations.  The set-up (STFT of every channel,
    filter-history allocation) is excluded, as it is on the GPU side."""
    from danse_amd.scene import make_scene
    from oracle import danse_ref_cpu as O
    K = len(M)
    sc = make_scene(M, sigDur=wl['dur'], seed=2000)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    b = O.BatchDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive)
    t = time.perf_counter()
    n = 0
    while n < K and (n == 0 or time.perf_counter() - t < seconds):
        b.batch_update_danse_covmats(n)
        b.perform_update(n)
        b.update_external_filters(n)
        b.batch_estimate(n)
        b.get_mmse_cost(n)
        n += 1
    tn = (time.perf_counter() - t) / n
    F = dp.DFTsize // 2 + 1
    nseg = b.yinSTFT[0].shape[1]
    iters = wl['iters']
    total = tn * K * iters
    cores, threads, env = _threads()
    return {'value': K * nseg * F * iters / total, 'unit': 'frame-updates/s', 'cores': threads, 'kind': 'port',
            'sample': f'float64 oracle batch DANSE (reference algorithm, per-bin scipy eigh), one process, default '
                      f'BLAS threads ({env or "no thread env set"}), scene seed 2000, iteration 1 of nodes 0..{n - 1} '
                      f'({tn:.2f} s per node), projected over {K} nodes x {iters} iterations: {total:.0f} s; host '
                      f'affinity {cores} cpus',
            't_node_s': tn, 'nodes_sampled': n, 'projected_run_s': total}


def pmc_traffic(wl, S, kernel_substr, rounds=None):
    """HBM bytes per launch of the dominant kernel from two rocprofv3 PMC
    passes over the same workload (MI355X_MICROARCH.md, HBM section):
    FETCH_SIZE and WRITE_SIZE (KiB) in separate passes, FETCH_SIZE doubled
    (gfx950 reports half the bytes of a wide streaming read).

    kernel_substr None: the per-round update group, exactly what the HIP
    events of run_online bracket (danse_engine_update: the class launches,
    the lean cached-C solves, their fallback launch, ff copies and the
    per-round estimators) -- in the un-graphed pass every dispatch between
    round r's bcast_kernel and round r + 1's, gate checks excluded; the
    counters are summed per round and averaged over the rounds mask.  The
    kernel mix of those rounds (dispatches per kernel) comes back with it."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which('rocprofv3')
    if exe is None:
        return None
    out = {}
    mix = None
    tmp = tempfile.mkdtemp(prefix='danse_pmc_')
    env = dict(os.environ, TMPDIR=os.environ.get('TMPDIR', '/tmp'))
    for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
        _progress(f'PMC pass {counter} ({wl["name"]})')
        d = os.path.join(tmp, counter)
        cmd = [exe, '--pmc', counter, '--kernel-trace', '-d', d, '-o', 'pmc', '--output-format', 'csv', '--',
               sys.executable, str(ROOT / 'bench.py'), '--pmc-child', '--workload', wl['name'], *_CHILD_ARGS,
               '--scenes', str(S)]
        try:
            subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, check=True)
        except Exception as e:   # profiler unavailable or refused: report null, never fail the bench
            return {'error': f'{counter}: {type(e).__name__}'}
        files = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith('counter_collection.csv')]
        rows = [row for fn in files for row in csv.DictReader(open(fn)) if row['Counter_Name'] == counter]
        if rows and 'Dispatch_Id' in rows[0]:
            rows.sort(key=lambda row: int(row['Dispatch_Id']))
        if kernel_substr is None:
            # group by round: a bcast_kernel dispatch opens each round
            groups, names, cur = [], [], None
            for row in rows:
                kn = row['Kernel_Name']
                if 'bcast_kernel' in kn:
                    cur = [0.0]
                    groups.append(cur)
                    names.append([])
                    continue
                if cur is None or 'gate_kernel' in kn or 'span_rec' in kn:
                    continue
                cur[0] += float(row['Counter_Value']) * 1024.0
                names[-1].append(kn.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '').strip())
            nR = len(rounds) if rounds is not None else len(groups) - 1
            if len(groups) < nR or nR == 0:
                return {'error': f'{counter}: {len(groups)} broadcast dispatches for {nR} rounds'}
            m = np.asarray(rounds, dtype=bool) if rounds is not None else np.ones(nR, dtype=bool)
            vals = np.array([g[0] for g in groups[:nR]])[m]
            if mix is None:
                mix = {}
                for r in np.nonzero(m)[0]:
                    for kn in names[r]:
                        mix[kn] = mix.get(kn, 0) + 1
        else:
            rows = [row for row in rows if kernel_substr in row['Kernel_Name']]
            if not rows:
                return {'error': f'{counter}: no samples'}
            vals = np.array([float(row['Counter_Value']) * 1024.0 for row in rows])
            # (one update dispatch per round in the un-graphed pass: the rounds
            # mask picks the solve rounds the roofline's duration is taken over)
            if rounds is not None and len(vals) == len(rounds):
                vals = vals[np.asarray(rounds, dtype=bool)]
        out[counter] = float(np.mean(vals))
        out['dispatches'] = int(len(vals))
    shutil.rmtree(tmp, ignore_errors=True)
    b = 2.0 * out['FETCH_SIZE'] + out['WRITE_SIZE']
    res = {'bytes_per_launch': b, 'fetch_bytes_raw': out['FETCH_SIZE'], 'write_bytes': out['WRITE_SIZE'],
           'dispatches': out['dispatches'], 'method': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, '
           'FETCH_SIZE x2 (gfx950)' + ('; summed over each round\'s update group (the HIP-event span), averaged '
                                       'over the same rounds' if kernel_substr is None else '')}
    if mix is not None:
        res['kernel_mix'] = dict(sorted(mix.items(), key=lambda kv: -kv[1]))
    return res


def ctypes_void(p):
    import ctypes
    return ctypes.c_void_p(p)


def _gate_rounds(sc, D):
    """Per node, the first round whose SCM counters pass the update gate
    (numUpdatesRyy > D and numUpdatesRnn > D): the oracle's startRound, which
    the engine reproduces exactly."""
    starts = []
    for nd in sc.wasn:
        v = nd.vadPerFrame
        ny = np.cumsum(v)
        nn = np.arange(1, len(v) + 1) - ny
        starts.append(int(np.argmax((ny > D) & (nn > D))))
    return np.array(starts)


def _threads():
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count()
    env = {k: os.environ[k] for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS')
           if k in os.environ}
    lim = [int(v) for v in env.values() if v.isdigit()]
    return cores, (min([cores] + lim) if lim else cores), env


def cpu_baseline(M, wl, dp, wp, seconds, rounds=None, seed=1000):
    """The float64 CPU oracle (oracle/danse_ref_cpu.py: the reference's
    per-frame NumPy/SciPy algorithm, per-bin scipy.linalg.eigh(Ryy, Rnn))
    timed on this host, one process, BLAS/OpenMP at their default threads
    (SURVEY §8d), on scene seed 1000 of the workload.

    value = whole-run frame-updates/s, the quantity the GPU line reports:
    K F R / (R t_round + sum_k (R - start_k) t_solve), with
      t_round = the oracle's measured per-round cost before any node passes
                its gate (WOLA, compression, both SCM recursions, estimate),
      t_solve = the measured per-node cost of a GEVD filter update over the
                F bins, start_k = node k's gate round (from the counters).
    Both come from bounded samples: t_round from the first rounds of the real
    run; t_solve from the real post-gate rounds when the gate opens within the
    time budget (config B: 'window'), otherwise from the oracle's own
    update_w_gevd over one node's F bins of Hermitian positive-definite pairs
    (N2: the K=32 x 8 gate opens at round 181 of a run costing ~0.6 s per
    round before it, 'solve sample').  Checked in the build container
    (DESIGN.md "CPU baseline"): the window projection is within 8% of the
    oracle's real whole run at K=8 x 4, and the solve sample under-prices a
    real K=32 x 8 post-gate round by 13% (15.5 s vs 17.8 s), so the N2 CPU
    rate is, if anything, over-stated."""
    from danse_amd.scene import make_scene
    from oracle import danse_ref_cpu as O
    sc = make_scene(M, sigDur=wl['dur'], seed=seed, SROperNode=wl.get('sros'))
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    K, F = len(M), dp.DFTsize // 2 + 1
    D = max(M) + K - 1
    starts = _gate_rounds(sc, D)
    R = rounds or (int((sc.wasn[0].data.shape[0] - dp.DFTsize) / dp.Ns) + 1)
    r0 = int(starts.min())
    kw = {}
    dxcp = getattr(dp, 'estimateSROs', 'Oracle') == 'DXCPPhaT'
    if dxcp:
        # the DANSE part with external (zero) SRO estimates; the DXCP-PhaT
        # estimators are timed on their own below (oracle/dxcp_ref.py)
        kw['sroEstimates'] = [np.zeros((R + 1, K - 1)) for _ in range(K)]
    # t_round: rounds 1..n of the real run (round 0 carries the set-up)
    npre = int(max(3, min(r0 - 1, 12)))
    probe = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive, maxRounds=npre + 1, **kw)
    probe.run()
    rt = probe.roundTimes
    t_round = (rt[-1][1] - rt[1][1]) / max(rt[-1][0] - rt[1][0], 1)
    # t_solve: a single-node GEVD over F bins from the oracle (used for the budget, and as the estimate
    # when the real post-gate window does not fit)
    rng = np.random.default_rng(0)

    def pd(n):
        Y = (rng.standard_normal((F, D, n)) + 1j * rng.standard_normal((F, D, n))) / np.sqrt(2 * n)
        return Y @ np.conj(np.swapaxes(Y, -1, -2))
    A, B = pd(4 * D), pd(4 * D)
    O.update_w_gevd(A[:8], B[:8], refSensorIdx=0, rank=1)
    t = time.perf_counter()
    nrep = 0
    while nrep < 1 or time.perf_counter() - t < 1.0:
        O.update_w_gevd(A, B, refSensorIdx=0, rank=1)
        nrep += 1
    t_solve_sample = (time.perf_counter() - t) / nrep
    rlast = int(starts.max())
    budget = rlast * t_round + 4 * (t_round + K * t_solve_sample)
    if budget <= 2.0 * seconds and R - rlast - 2 >= 1:
        nwin = int(max(1, min(R - rlast - 2, seconds / max(t_round + K * t_solve_sample, 1e-3))))
        # (the window skips the gate round itself, whose Hermitian/PSD/rank check costs one more eigh)
        ov = O.OnlineDANSE(sc, dp, vadMinProp=wp.vadMinProportionActive, maxRounds=rlast + 1 + nwin, **kw)
        ov.run()
        rt = dict(ov.roundTimes)
        t_post = (rt[rlast + 1 + nwin] - rt[rlast + 1]) / nwin
        t_solve = (t_post - t_round) / K
        method = f'window: rounds 1..{npre} (t_round) and {rlast + 1}..{rlast + 1 + nwin} (all nodes past the gate)'
        sampled = rt[rlast + nwin] - rt[min(rt)]
    else:
        t_solve = t_solve_sample
        method = (f'solve sample: rounds 1..{npre} of the real run (t_round) + the oracle update_w_gevd over '
                  f'{F} bins x D={D} ({nrep} reps)')
        sampled = rt[-1][1] - rt[0][1] + t_solve * nrep
    total = R * t_round + float(np.sum(np.maximum(R - starts, 0))) * t_solve
    if dxcp:
        # DXCP-PhaT (the reference's DXCPPhaT class, restated): one estimator
        # per (receiver, sender), fed a 2048-sample block every 4 rounds
        from oracle import dxcp_ref as X
        est = X.DXCPPhaT()
        rng = np.random.default_rng(0)
        blk = rng.standard_normal((X.FRAME, 2))
        for _ in range(8):
            est.process_data(blk)
        t = time.perf_counter()
        nb = 0
        while nb < 8 or time.perf_counter() - t < 1.0:
            est.process_data(blk)
            nb += 1
        t_dx = (time.perf_counter() - t) / nb
        nfed = R * dp.Ns // X.FRAME
        total += K * (K - 1) * nfed * t_dx
        method += f'; DXCP-PhaT {K * (K - 1)} estimators x {nfed} blocks at {t_dx * 1e3:.2f} ms per block'
    cores, threads, env = _threads()
    return {'value': K * F * R / total, 'unit': 'frame-updates/s', 'cores': threads, 'kind': 'port',
            'sample': f'float64 oracle (reference algorithm, per-bin scipy eigh), one process, default BLAS threads '
                      f'({env or "no thread env set"}), scene seed {seed}, {method}; {sampled:.1f} s sampled; '
                      f'whole run projected over {R} rounds: {total:.1f} s; host affinity {cores} cpus',
            't_round_s': t_round, 't_solve_node_s': t_solve, 't_solve_sample_s': t_solve_sample,
            'gate_rounds': [int(starts.min()), int(starts.max())], 'projected_run_s': total}


if __name__ == '__main__':
    main()
