"""Case definitions shared by ``make_golden.py`` (reference side, build
container only) and the tests (no reference import).  Each case names the
reference configuration it mirrors."""
from __future__ import annotations

import numpy as np

# sandbox YAML (config A) settings, config_files/sandbox_config.yaml:13-80
SANDBOX = dict(simType='online', performGEVD=True, use1stFrameAsBasis=True,
               filterInitType='fixedValue', filterInitFixedValue=1,
               forcedBetaExternalFilters=0.7, t_expAvg50p=1, t_expAvg50pExternalFilters=1,
               startComputeMetricsAt='after_200ms', covMatInitType='fully_random')
# battery YAML (configs B-E), config_files/sandbox_config_battery20230919.yaml
BATTERY = dict(simType='online', performGEVD=True, use1stFrameAsBasis=True,
               filterInitType='selectFirstSensor', forcedBetaExternalFilters=0.7,
               t_expAvg50p=1, t_expAvg50pExternalFilters=1, startComputeMetricsAt='after_200ms',
               noFusionAtSingleSensorNodes=True)


def _d(base, **kw):
    out = dict(base)
    out.update(kw)
    return out


ONLINE_CASES = [
    # config A shape: K=2 x 1 mic, seq, GEVD r1, local + centralised + SSBC, SNR replay
    dict(name='online_A_k2m1_seq', M=[1, 1], dur=2.0, seed=1, snr_replay=True,
         danse=_d(SANDBOX, nodeUpdating='seq', computeLocal=True, computeCentralised=True,
                  computeSingleSensorBroadcast=True)),
    # config B shape (smaller K): asy GEVD r1, battery settings
    dict(name='online_B_k4m3_asy', M=[3, 3, 3, 3], dur=2.0, seed=2,
         danse=_d(BATTERY, nodeUpdating='asy')),
    dict(name='online_B_k4m3_seq', M=[3, 3, 3, 3], dur=2.0, seed=2,
         danse=_d(BATTERY, nodeUpdating='seq')),
    # ragged nodes, GEVD rank 2, local + centralised, asy
    dict(name='online_ragged_asy_r2', M=[2, 3, 2], dur=2.0, seed=3,
         danse=_d(SANDBOX, nodeUpdating='asy', GEVDrank=2, computeLocal=True, computeCentralised=True)),
    # MWF (no GEVD), seq and asy; no first-frame basis (eps-random SCM init path)
    dict(name='online_mwf_seq', M=[2, 2], dur=2.0, seed=4,
         danse=_d(SANDBOX, nodeUpdating='seq', performGEVD=False)),
    dict(name='online_mwf_asy_nobasis', M=[2, 2, 2], dur=2.0, seed=5,
         danse=_d(BATTERY, nodeUpdating='asy', performGEVD=False, use1stFrameAsBasis=False)),
    # GEVD without the first-frame basis: the SCMs start from the eps-scaled
    # random init (d_base.py:2446-2450, non-Hermitian; eigh reads the lower triangle)
    dict(name='online_gevd_asy_nobasis', M=[2, 3, 2], dur=2.0, seed=12,
         danse=_d(BATTERY, nodeUpdating='asy', use1stFrameAsBasis=False)),
    # init variants (d_base.py:2367-2470, d_classes.py:553-700): random filters
    # (seed 0 over the whole (F, nIter + 1, D) history), per-bin and per-node
    # eye + eps-scaled random SCMs (non-Hermitian at eps scale; eigh reads the
    # lower triangle), no first-frame basis so the init stays in the recursion
    dict(name='online_init_random_asy', M=[2, 3, 2], dur=2.0, seed=13,
         danse=_d(BATTERY, nodeUpdating='asy', filterInitType='random', covMatInitType='eye_and_random',
                  covMatSameInitForAllFreqs=False,
                  covMatSameInitForAllNodes=False, use1stFrameAsBasis=False, computeLocal=True,
                  computeCentralised=True)),
    # the reference gate delays the start (check_covariance_matrices,
    # d_classes.py:1430-1540): a 1e-6 non-Hermitian init residue decays with
    # beta^m until np.allclose(X^H, X) holds -- nodes start at iterations 29,
    # 28 and 54 although the frame counters allow 26
    dict(name='online_gate_delay_asy', M=[2, 2, 2], dur=3.0, seed=14,
         danse=_d(BATTERY, nodeUpdating='asy', covMatInitType='eye_and_random', covMatRandomInitScaling=1e-6,
                  use1stFrameAsBasis=False, t_expAvg50p=0.1)),
    # config C shape (fewer nodes): SROs, Oracle SRO estimates, phase compensation with
    # full-sample-drift flags (d_classes.py:1936-2046, 2364-2621; quirks Q3, Q5, Q13)
    dict(name='online_C_sro_comp_asy', M=[2, 3, 2], dur=3.0, seed=8, sros=[0, 100, 200],
         danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=True, includeFSDflags=True, estimateSROs='Oracle',
                  computeLocal=True)),
    # CohDrift SRO estimation (d_sros.py:19-95, d_classes.py:2364-2621): closed
    # loop, least-squares fit over bins, estimates feeding the phase
    # compensation from iteration startAfterNups + estEvery on
    dict(name='online_C_cohdrift_asy', M=[2, 3, 2], dur=3.0, seed=15, sros=[0, 60, 120],
         danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=True, includeFSDflags=True, estimateSROs='CohDrift',
                  cohDrift=dict(estimationMethod='ls'))),
    # the open loop (cohDrift.loop 'open', d_classes.py:2439-2450,2580-2584):
    # the coherence of the UNcompensated observation, the residual phase
    # corrected by the full-sample-drift flags of the last segLength rounds
    # (d_sros.py:19-95), the residual itself as the estimate
    dict(name='online_C_cohdrift_open_asy', M=[2, 3, 2], dur=3.0, seed=15, sros=[0, 60, 120],
         danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=True, includeFSDflags=True, estimateSROs='CohDrift',
                  cohDrift=dict(estimationMethod='ls', loop='open'))),
    # CohDrift under sequential node updating (closed loop)
    dict(name='online_C_cohdrift_seq', M=[2, 2, 3], dur=3.0, seed=23, sros=[0, 80, 160],
         danse=_d(BATTERY, nodeUpdating='seq', compensateSROs=True, includeFSDflags=True, estimateSROs='CohDrift',
                  cohDrift=dict(estimationMethod='ls'))),
    dict(name='online_C_sro_noflags_seq', M=[2, 2, 2, 2], dur=3.0, seed=9, sros=[50, 0, 200, 120],
         danse=_d(BATTERY, nodeUpdating='seq', compensateSROs=True, includeFSDflags=False, estimateSROs='Oracle')),
    # config E shape (tests/battery20230919_perf_asfctofL.py:14-110): MK = [2, 3],
    # broadcastType 'fewSamples' with efficientSpSBC (T(z) compression, L-sample
    # broadcasts, IR refresh every upTDfilterEvery = 1 s; d_classes.py:1090-1160,
    # d_base.py:837-863, 1871-1991); 2.5 s so the IR is refreshed twice
    dict(name='online_E_fs_L64_asy', M=[2, 3], dur=2.5, seed=10,
         danse=_d(BATTERY, nodeUpdating='asy', broadcastType='fewSamples', broadcastLength=64,
                  computeLocal=True, computeCentralised=True)),
    dict(name='online_E_fs_L128_sro_comp', M=[2, 3], dur=2.5, seed=11, sros=[0, 200],
         danse=_d(BATTERY, nodeUpdating='asy', broadcastType='fewSamples', broadcastLength=128,
                  compensateSROs=True, includeFSDflags=True, estimateSROs='Oracle', computeLocal=True)),
    # the E battery's settings (tests/battery20230919_perf_asfctofL.py:60-104):
    # local, centralised and single-sensor-broadcast estimates under SRO clocks.
    # Centralised buffers carry raw signals through the same buffers as z
    # (fill_buffers_centr / process_incoming_signals_buffers_centr,
    # d_classes.py:1226-1250,1809-1891); their compensation uses the flag index
    # arithmetic of compensate_sros (d_classes.py:2000-2038, quirk Q14).  SSBC
    # with compensation raises in the reference (d_classes.py:2042-2044).
    dict(name='online_C_sro_centr_asy', M=[2, 3, 2], dur=3.0, seed=16, sros=[0, 100, 200],
         danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=True, includeFSDflags=True, estimateSROs='Oracle',
                  computeLocal=True, computeCentralised=True)),
    dict(name='online_C_sro_ssbc_nocomp_asy', M=[1, 2, 3], dur=3.0, seed=17, sros=[0, 150, 300],
         danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=False, estimateSROs='Oracle',
                  computeLocal=True, computeCentralised=True, computeSingleSensorBroadcast=True)),
    dict(name='online_E_fs_L64_sro_nocomp', M=[2, 3], dur=2.5, seed=18, sros=[0, 200],
         danse=_d(BATTERY, nodeUpdating='asy', broadcastType='fewSamples', broadcastLength=64,
                  compensateSROs=False, estimateSROs='Oracle', computeLocal=True, computeCentralised=True,
                  computeSingleSensorBroadcast=True)),
    dict(name='online_E_fs_L256_sro_comp_centr', M=[2, 3], dur=2.5, seed=19, sros=[0, 200],
         danse=_d(BATTERY, nodeUpdating='asy', broadcastType='fewSamples', broadcastLength=256,
                  compensateSROs=True, includeFSDflags=True, estimateSROs='Oracle', computeLocal=True,
                  computeCentralised=True)),
    dict(name='online_E_fs_L1_seq', M=[2, 3, 1], dur=2.5, seed=12,
         danse=_d(BATTERY, nodeUpdating='seq', broadcastType='fewSamples', broadcastLength=1)),
    # the E battery's remaining broadcast lengths under SROs [0, 200] ppm
    # (tests/battery20230919_perf_asfctofL.py:21-24,60-104): L < 32 puts the
    # faster node's chunk after its own update (with the next iteration's IR
    # at the refresh timer), L = Ns broadcasts twice in iteration 0
    # (scheduler.compile_rounds_fs step lists)
    *[dict(name=f'online_E_fs_L{L}_sro_{tag}', M=[2, 3], dur=dur, seed=seed, sros=[0, 200],
           danse=_d(BATTERY, nodeUpdating='asy', broadcastType='fewSamples', broadcastLength=L,
                    compensateSROs=comp, includeFSDflags=comp, estimateSROs='Oracle', computeLocal=True,
                    computeCentralised=True, computeSingleSensorBroadcast=not comp))
      for L, dur, seed in ((1, 2.5, 20), (16, 6.0, 21), (512, 2.5, 22))
      for tag, comp in (('nocomp', False), ('comp', True))],
    # desSigProcessingType 'conv': T(z) time-domain estimates of every family
    # (get_desired_sig_chunk, d_base.py:2085-2100), ragged nodes, asy
    dict(name='online_conv_ragged_asy', M=[2, 3, 2], dur=2.0, seed=7,
         danse=_d(SANDBOX, nodeUpdating='asy', computeLocal=True, computeCentralised=True,
                  computeSingleSensorBroadcast=True, desSigProcessingType='conv')),
]

BATCH_CASES = [
    # d_batch: non frame-aligned length (quirk Q9)
    dict(name='batch_k3m2_asy', M=[2, 2, 2], dur=2.01, seed=6,
         danse=_d(BATTERY, simType='batch', nodeUpdating='asy', maxBatchUpdates=5)),
    dict(name='batch_k3_seq_mwf', M=[1, 2, 3], dur=2.01, seed=7,
         danse=_d(BATTERY, simType='batch', nodeUpdating='seq', maxBatchUpdates=4, performGEVD=False)),
    # random filter init: slot 0 of the reference's (F, nIter + 1, D) seed-0 draw
    dict(name='batch_k3_random_init_asy', M=[2, 3, 2], dur=2.01, seed=8,
         danse=_d(BATTERY, simType='batch', nodeUpdating='asy', maxBatchUpdates=4, filterInitType='random')),
    # centralised and local batch estimates (get_centralized_and_local_estimates,
    # d_batch.py:20-88; d_core.py:282-283)
    dict(name='batch_k3_local_centr_asy', M=[2, 3, 2], dur=2.01, seed=25,
         danse=_d(BATTERY, simType='batch', nodeUpdating='asy', maxBatchUpdates=3, computeLocal=True,
                  computeCentralised=True)),
]

# best-performance reference (d_core.get_best_perf, d_core.py:602-627: batch
# centralised estimates without SROs), on the online parameters of a case; the
# noise-only / speech-only replays with the recorded wCentr
# (generate_signals_for_snr_computation, d_core.py:550-599)
BESTPERF_CASES = [
    dict(name='bestperf_k3', M=[2, 3, 2], dur=2.01, seed=26, danse=_d(BATTERY, nodeUpdating='asy')),
    dict(name='bestperf_k4_mwf', M=[1, 2, 2, 3], dur=2.01, seed=27,
         danse=_d(SANDBOX, nodeUpdating='seq', performGEVD=False)),
]

SRO_EVENT_CASES = [
    dict(name='events_sro_0_50_100_seq', M=[1, 1, 1], dur=4.0, sros=[0, 50, 100],
         danse=_d(BATTERY, nodeUpdating='seq')),
    dict(name='events_sro_0_100_200_asy', M=[1, 1, 1], dur=4.0, sros=[0, 100, 200],
         danse=_d(BATTERY, nodeUpdating='asy')),
    dict(name='events_sro_0_0_seq', M=[2, 2], dur=3.0, sros=[0, 0],
         danse=_d(BATTERY, nodeUpdating='seq')),
]

KAT_CASES = [dict(name=f'kat_{"gevd" if g else "mwf"}_D{D}_r{r}', D=D, F=48, gevd=g, rank=r, ref=0, seed=100 + D + r)
             for (D, g, r) in [(2, True, 1), (11, True, 1), (11, True, 2), (19, True, 1), (39, True, 1),
                               (2, False, 1), (11, False, 1), (39, False, 1)]]
# the wide classes (64 < D <= 256: centralised estimates at sum(M) up to 256;
# kat_inputs takes ~25 s at D = 256, F = 8)
KAT_CASES += [dict(name=f'kat_{"gevd" if g else "mwf"}_D{D}_r{r}', D=D, F=F, gevd=g, rank=r, ref=ref, seed=100 + D + r)
              for (D, g, r, F, ref) in [(96, True, 1, 48, 0), (96, True, 2, 48, 5), (256, True, 1, 8, 0),
                                        (96, False, 1, 48, 3), (256, False, 1, 8, 0)]]


def kat_inputs(case):
    """Exponentially averaged rank-1 updates (the online SCM recursion,
    ``d_classes.py:2086-2090``) from a random mixing: Ryy has a strong
    rank-1 component over a spatially coloured noise floor."""
    rng = np.random.default_rng(case['seed'])
    F, D = case['F'], case['D']
    beta = 0.978063
    A = rng.standard_normal((F, D, D)) + 1j * rng.standard_normal((F, D, D))
    a = rng.standard_normal((F, D)) + 1j * rng.standard_normal((F, D))
    Rnn = np.zeros((F, D, D), dtype=complex)
    Ryy = np.zeros((F, D, D), dtype=complex)
    for t in range(3 * D + 10):
        n = np.einsum('fij,fj->fi', A, rng.standard_normal((F, D)) + 1j * rng.standard_normal((F, D)))
        s = a * (rng.standard_normal((F, 1)) + 1j * rng.standard_normal((F, 1))) * 3.0
        nn = 1 / D * np.einsum('ij,ik->ijk', n, n.conj())
        yy = 1 / D * np.einsum('ij,ik->ijk', n + s, (n + s).conj())
        Rnn = beta * Rnn + (1 - beta) * nn
        n2 = np.einsum('fij,fj->fi', A, rng.standard_normal((F, D)) + 1j * rng.standard_normal((F, D)))
        yy = 1 / D * np.einsum('ij,ik->ijk', n2 + s, (n2 + s).conj())
        Ryy = beta * Ryy + (1 - beta) * yy
    return Ryy, Rnn


# DXCP-PhaT sampling-rate-offset estimator (dxcpphat/sro_estimation.py,
# DXCPPhaT with default parameters): two channels of one band-limited
# multi-sine source, channel 2 sampled at (1 + sro 1e-6) fs with a delay.
DXCP_CASES = [
    dict(name='dxcp_sro100', dur=14.0, sro=100.0, delay=3.5, seed=31),
    dict(name='dxcp_sro_m60', dur=12.0, sro=-60.0, delay=-7.25, seed=32),
    dict(name='dxcp_sro200', dur=10.0, sro=200.0, delay=0.0, seed=33),
]


# closed-loop DXCP-PhaT (CL_DXCPPhaT, sro_estimation.py:12-72): online
# resampler + delay buffer + DXCP-PhaT + IMC controller; acsEvery > 0 sets
# acs = 0 on every acsEvery-th frame
CLDXCP_CASES = [
    dict(name='cldxcp_sro100', dur=40.0, sro=100.0, delay=3.5, seed=34, startDelay=0, acsEvery=0),
    dict(name='cldxcp_sro_m60', dur=30.0, sro=-60.0, delay=-2.0, seed=35, startDelay=12, acsEvery=7),
]


def cldxcp_acs(case, n):
    a = np.ones(n, dtype=np.int64)
    if case['acsEvery'] > 0:
        a[::case['acsEvery']] = 0
    return a


def dxcp_inputs(case, fs=16000.0):
    """Exact evaluation of a random multi-sine at each channel's sample
    instants (no resampler needed), plus independent sensor noise."""
    rng = np.random.default_rng(case['seed'])
    n = int(case['dur'] * fs)
    f = rng.uniform(100.0, 7000.0, 120)
    a = rng.uniform(0.2, 1.0, 120)
    ph = rng.uniform(0.0, 2 * np.pi, 120)
    t1 = np.arange(n) / fs
    t2 = (np.arange(n) * (1.0 + case['sro'] * 1e-6) + case['delay']) / fs
    x1 = np.zeros(n)
    x2 = np.zeros(n)
    for i in range(120):
        x1 += a[i] * np.cos(2 * np.pi * f[i] * t1 + ph[i])
        x2 += a[i] * np.cos(2 * np.pi * f[i] * t2 + ph[i])
    x1 += 0.05 * rng.standard_normal(n)
    x2 += 0.05 * rng.standard_normal(n)
    return x1.astype(np.float32).astype(np.float64), x2.astype(np.float32).astype(np.float64)


# T(z) few-samples compression KATs: dist_fct_approx +
# danse_compression_few_samples on seeded filters / frames.  'win' picks the
# analysis / synthesis windows: 'sqrthann' (the default DANSE windows) or
# 'rand' (independent positive random windows: exercises the asymmetric
# window correlation).  'update' False feeds the Dirac initial IR of
# d_classes.py:660-663 as wIRprevious.
TZ_CASES = [
    dict(name='tz_m2_L64', M=2, L=64, N=1024, Ns=512, win='sqrthann', update=True, seed=41),
    dict(name='tz_m3_L512', M=3, L=512, N=1024, Ns=512, win='sqrthann', update=True, seed=42),
    dict(name='tz_m1_L1', M=1, L=1, N=1024, Ns=512, win='rand', update=True, seed=43),
    dict(name='tz_m4_L128_dirac', M=4, L=128, N=1024, Ns=512, win='sqrthann', update=False, seed=44),
]


def tz_inputs(case):
    """(wHat [N/2+1, M] complex, yq [N, M], h, f, wIRprevious [2N-1, M])."""
    rng = np.random.default_rng(case['seed'])
    N, M = case['N'], case['M']
    F = N // 2 + 1
    wHat = rng.standard_normal((F, M)) + 1j * rng.standard_normal((F, M))
    yq = rng.standard_normal((N, M))
    if case['win'] == 'sqrthann':
        h = np.sqrt(np.hanning(N))
        f = h.copy()
    else:
        h = rng.uniform(0.1, 1.0, N)
        f = rng.uniform(0.1, 1.0, N)
    wPrev = np.zeros((2 * N - 1, M))
    wPrev[N, 0] = 1.0
    return wHat, yq, h, f, wPrev


# online cases whose schedule-derived dv fields (SRO estimates / residuals,
# flag iterations, first-update instant, MSE-cost arrays) and whole-signal
# STFTs (yinSTFT, bins subsampled) are dumped as fields_<case>.npz
# enhancement metrics (d_eval.py get_snr / get_fwsnrseg): seeded signals
METRIC_CASES = [
    dict(name='metrics_fw_16k', T=16000, fs=16000.0, seed=301, noise=0.3, same=0),
    dict(name='metrics_fw_ragged', T=24037, fs=16000.0, seed=302, noise=0.05, same=4000),
    dict(name='metrics_fw_8k_frame20', T=12011, fs=8000.0, seed=303, noise=1.0, same=0, frameLen=0.02,
         overlap=0.5, gamma=0.3),
]


def metric_inputs(case):
    """clean: bursts of low-passed noise (speech-like on/off); enhanced: the
    clean signal scaled, plus noise, identical to it over the first `same`
    samples (exercises the eps clamp and the 35 dB clip); s / n / vad for
    get_snr: [T x 3]."""
    rng = np.random.default_rng(case['seed'])
    T = case['T']
    x = rng.standard_normal(T)
    x = np.convolve(x, np.ones(8) / 8, mode='same')
    env = (np.sin(2 * np.pi * np.arange(T) / 3000.0) > -0.2).astype(float)
    clean = x * env
    enh = 0.8 * clean + case['noise'] * rng.standard_normal(T)
    enh[:case['same']] = clean[:case['same']]
    s = rng.standard_normal((T, 3)) * np.array([1.0, 0.5, 2.0])
    n = rng.standard_normal((T, 3)) * np.array([0.3, 0.7, 1.5])
    vad = (rng.random((T // 100 + 1, 3)) > 0.4).repeat(100, axis=0)[:T]
    return clean, enh, s, n, vad


# get_metrics ('snr', 'fwSNRseg' entries) on seeded DANSE-like outputs
GETMETRICS_CASE = dict(name='metrics_get_metrics', T=32000, fs=16000.0, seed=311, startIdx=2000, endIdx=30500)


def get_metrics_inputs(case):
    rng = np.random.default_rng(case['seed'])
    T = case['T']
    x = np.convolve(rng.standard_normal(T), np.ones(6) / 6, mode='same')
    env = (np.sin(2 * np.pi * np.arange(T) / 4000.0) > -0.3).astype(float)
    clean = x * env
    noise = 0.5 * rng.standard_normal(T)
    kw = dict(clean=clean, noiseOnly=noise, noisy=clean + noise,
              filtSpeech=0.9 * clean + 0.02 * rng.standard_normal(T), filtNoise=0.1 * noise,
              filtSpeech_c=0.95 * clean, filtNoise_c=0.05 * noise, filtSpeech_l=0.8 * clean, filtNoise_l=0.3 * noise)
    kw['enhan_c'] = kw['filtSpeech_c'] + kw['filtNoise_c']
    kw['enhan_l'] = kw['filtSpeech_l'] + kw['filtNoise_l']
    kw['vad'] = env.astype(bool)
    return kw


FIELD_CASES = ['online_C_sro_comp_asy', 'online_C_sro_noflags_seq', 'online_B_k4m3_seq', 'online_ragged_asy_r2',
               'online_E_fs_L64_asy', 'online_C_cohdrift_open_asy', 'online_C_cohdrift_seq']
FIELD_STFT_BIN_STEP = 37


# (e)STOI (danse_toolbox/mypystoi/stoi.py): at 10 kHz stoi_any_fs (no
# resampling; resampy is absent offline), at 16 kHz stoi() (the Octave
# resampler utils.resample_oct, scipy); extended (eSTOI, what get_metrics
# uses, d_eval.py:254-331) and classic
STOI_CASES = [
    dict(name='stoi_10k', T=60000, fs=10000, seed=401, noise=0.4, fn='stoi_any_fs'),
    dict(name='stoi_16k_oct', T=96000, fs=16000, seed=402, noise=0.25, fn='stoi'),
    dict(name='stoi_16k_oct_ragged', T=80123, fs=16000, seed=403, noise=1.0, fn='stoi'),
]


def stoi_inputs(case):
    """clean: on/off bursts of coloured noise with silent stretches (the
    silent-frame removal drops them); enhanced: scaled clean plus noise."""
    rng = np.random.default_rng(case['seed'])
    T = case['T']
    x = rng.standard_normal(T)
    x = np.convolve(x, np.ones(6) / 6, mode='same')
    env = (np.sin(2 * np.pi * np.arange(T) / (0.7 * case['fs'])) > 0.1).astype(float)
    env *= 0.5 + 0.5 * np.abs(np.sin(2 * np.pi * np.arange(T) / (0.13 * case['fs'])))
    clean = x * env
    enh = 0.7 * clean + case['noise'] * np.convolve(rng.standard_normal(T), np.ones(3) / 3, mode='same')
    return clean, enh


# end to end: the reference's online DANSE, its noise-only / speech-only
# replays (generate_signals_for_snr_computation, d_core.py:550-599) and
# get_metrics (d_eval.py:70-373; snr and fwSNRseg -- its stoi needs resampy)
# per node, from sample startIdx to the end
E2E_METRICS_CASE = dict(name='metrics_e2e_k3', M=[2, 2, 2], dur=4.0, seed=31, startIdx=16000,
                        danse=_d(BATTERY, nodeUpdating='asy', computeLocal=True, computeCentralised=True))


# The device scene generator's convolution and VAD (csrc/scene.hip) against
# the reference's own get_vad (siggen/utils.py:834-893: wet signals by
# sig.fftconvolve(xdry, rir)[:N], oracleVAD on each node's reference sensor,
# utils.py:896-939,1079-1151) on injected inputs: a paused uniform dry source
# and uniform random IRs (float32 values), stored in the fixture.
SCENE_CASES = [dict(name='scene_vad_conv', M=[2, 1, 2], T=32000, nIR=3200, seed=5, fs=16000.0,
                    vadWinLength=0.04, vadEnergyDecrease_dB=40.0)]


def scene_inputs(case):
    """(xdry [T], IRs [sum M][nIR]) as float32-valued float64 arrays."""
    rng = np.random.default_rng(case['seed'])
    T, fs = case['T'], case['fs']
    x = rng.uniform(-1, 1, T).astype(np.float32).astype(np.float64)
    t = np.arange(T) / fs
    x[np.fmod(t, 1.0) >= 0.5] = 0.0
    h = (0.5 * rng.uniform(-1, 1, (sum(case['M']), case['nIR']))).astype(np.float32).astype(np.float64)
    return x, h


# Condition numbers (saveConditionNumber: ConditionNumbers.get_new_cond_number,
# d_classes.py:19-130,2126-2186) from the reference's own online run: the
# shape of tests/test_gpu_engine_modes.py::test_condition_numbers_vs_oracle.
COND_CASES = [dict(name='cond_k4m3', M=[3, 3, 3, 3], dur=2.0, seed=41,
                   danse=_d(BATTERY, nodeUpdating='asy', computeLocal=True, saveConditionNumber=True,
                            saveConditionNumberEvery=3))]


# online modes whose error behaviour is pinned (make_golden._run_modes):
# covMatInitType 'batch_estimates' raises inside the reference itself
# (init_covmats_from_batch, d_classes.py:1002-1005)
REF_MODES_CASE = dict(name='ref_modes', base=BATTERY,
                      modes={'batch_estimates': dict(covMatInitType='batch_estimates')})
