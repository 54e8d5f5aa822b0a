"""HIP path (through the C-ABI) against the CPU oracle and the reference's
golden vectors.  Runs on an MI355X only (``-m gpu``).

Tolerances (fp32 complex device arithmetic vs the float64 reference):
* filters w: per-bin relative error ||w_gpu - w_ref|| / ||w_ref|| over all
  bins, nodes and compared iterations: median <= 1e-5 and 99th percentile
  <= 1e-4 (the north-star "rel. err <= 1e-4 on filters", stated as a
  percentile as SURVEY §8c recommends: isolated ill-conditioned bins are
  reported, not hidden);
* time-domain estimates d: ||d_gpu - d_ref|| / ||d_ref|| <= 1e-4;
* integer/boolean state (gating round, number of filter updates): exact.
"""
import ctypes

import numpy as np
import pytest

from golden_cases import ONLINE_CASES, BATCH_CASES, KAT_CASES, kat_inputs, BESTPERF_CASES
from _util import make_case_params, make_case_scene, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')


def _lib():
    from danse_amd import _lib as L
    return L, L.load_library()


def _dev_cf(a):
    t = torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.complex64)).view(np.float32)).cuda()
    return t


def _bin_rel(w, wr):
    num = np.linalg.norm(w - wr, axis=-1)
    den = np.linalg.norm(wr, axis=-1)
    return num / np.maximum(den, 1e-30)


def _lapack_fp32_filters(Ryy, Rnn, case):
    import scipy.linalg as sla
    out = []
    for f in range(Ryy.shape[0]):
        A, B = Ryy[f].astype(np.complex64), Rnn[f].astype(np.complex64)
        if not case['gevd']:   # same factorisation as the kernel: Cholesky of Ryy
            out.append(sla.cho_solve(sla.cho_factor(A, lower=True), (A - B)[:, case['ref']]))
            continue
        s, X = sla.eigh(A, B)
        idx = np.argsort(s)[::-1]
        s, X = s[idx], X[:, idx]
        R = case['rank']
        Q = np.linalg.inv(X.conj().T)
        out.append((X[:, :R] @ np.diag(1 - 1 / s[:R]) @ Q[:, :R].conj().T)[:, case['ref']])
    return np.array(out, dtype=np.complex128)


def _stats(e):
    e = np.asarray(e).ravel()
    return dict(median=float(np.median(e)), p99=float(np.percentile(e, 99)), max=float(e.max()))


@pytest.mark.parametrize('case', KAT_CASES, ids=lambda c: c['name'])
def test_filter_update_kat(case, golden_dir):
    L, lib = _lib()
    g = np.load(golden_dir / f"{case['name']}.npz")
    Ryy, Rnn = kat_inputs(case)
    F, D = case['F'], case['D']
    a = torch.from_numpy(np.ascontiguousarray(np.asarray(Ryy, dtype=np.complex128)).view(np.float64)).cuda()
    n = torch.from_numpy(np.ascontiguousarray(np.asarray(Rnn, dtype=np.complex128)).view(np.float64)).cuda()
    w = torch.empty((F, D, 2), dtype=torch.float32, device='cuda')
    diag = torch.zeros(F, dtype=torch.int32, device='cuda')
    L.check(lib.danse_filter_update(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(n.data_ptr()), F, D,
                                    int(case['gevd']), case['rank'], case['ref'], ctypes.c_void_p(w.data_ptr()),
                                    ctypes.c_void_p(diag.data_ptr()), None))
    torch.cuda.synchronize()
    wg = w.cpu().numpy().view(np.complex64)[..., 0].astype(np.complex128)
    e = _bin_rel(wg, g['w'])
    st = _stats(e)
    # for scale: LAPACK in single precision (Cholesky solve for MWF,
    # generalized eigensolver for GEVD) on the same inputs; the device's
    # mixed-precision update (float64 factorisation of Rnn) beats it and is
    # held to the north-star tolerance itself
    try:
        st32 = _stats(_bin_rel(_lapack_fp32_filters(Ryy, Rnn, case), g['w']))
    except np.linalg.LinAlgError:   # (single-precision LAPACK: Rnn not positive definite at D = 256)
        st32 = None
    print(case['name'], st, 'lapack-fp32', st32)
    assert int(diag.sum()) == 0
    assert st['median'] <= 1e-5 and st['p99'] <= 1e-4, (st, st32)


def test_wola_analysis_matches_numpy():
    L, lib = _lib()
    rng = np.random.default_rng(0)
    C, T, N, Ns = 7, 5000, 1024, 512
    x = rng.uniform(-1, 1, (C, T)).astype(np.float32)
    ends = np.array([512, 1024, 1536, 3000, 4999, 5000, 700], dtype=np.int32)
    win = np.sqrt(np.hanning(N)).astype(np.float32)
    xd, ed, wd = torch.from_numpy(x).cuda(), torch.from_numpy(ends).cuda(), torch.from_numpy(win).cuda()
    out = torch.empty((C, N // 2 + 1, 2), dtype=torch.float32, device='cuda')
    L.check(lib.danse_wola_analysis(ctypes.c_void_p(xd.data_ptr()), C, T, ctypes.c_void_p(ed.data_ptr()),
                                    ctypes.c_void_p(wd.data_ptr()), N, Ns, ctypes.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.complex64)[..., 0]
    for c in range(C):
        fr = np.zeros(N)
        b = max(ends[c] - N, 0)
        seg = x[c, b:ends[c]].astype(np.float64)
        fr[N - len(seg):] = seg
        ref = np.fft.fft(fr * win.astype(np.float64))[:N // 2 + 1] / np.sqrt(Ns)
        assert rel_err(got[c], ref) < 2e-6


def _compare_online(case, dv, ov, label=''):
    K = len(case['M'])
    errs = []
    for k in range(K):
        s0 = int(ov.startRound[k])
        R = dv.nRounds
        # compare iterations after the node started updating
        wg = dv.wTilde[k][:, s0 + 1:R + 1, :]
        wr = ov.wTilde[k][:, s0 + 1:R + 1, :]
        errs.append(_bin_rel(wg, wr).ravel())
    st = _stats(np.concatenate(errs))
    de = rel_err(dv.d, ov.d)
    print(label, case['name'], 'w', st, 'd', de)
    return st, de


@pytest.mark.parametrize('case', ONLINE_CASES, ids=lambda c: c['name'])
def test_online_engine_vs_oracle(case, golden_dir):
    from danse_amd.core import danse_multi
    from oracle import danse_ref_cpu as O
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    dv = danse_multi([sc], dp)[0]
    ov = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive)
    # exact integer state
    assert np.array_equal(dv.startRound, ov.startRound)
    assert np.array_equal(dv.nInternalFilterUps, ov.nInternalFilterUps)
    assert int(np.sum(dv.diag)) == 0
    st, de = _compare_online(case, dv, ov)
    flags = {'dLocal': 'computeLocal', 'dCentr': 'computeCentralised', 'dSSBC': 'computeSingleSensorBroadcast'}
    for nm, fl in flags.items():
        if case['danse'].get(fl, False):
            e = rel_err(getattr(dv, nm), getattr(ov, nm))
            print('  ', nm, e)
            assert e <= 1e-4, (nm, e)
    # the other families' filter histories (local / centralised / SSBC;
    # under SRO clocks the centralised vector's raw frames and compensation)
    for wn, fl in (('wLocal', 'computeLocal'), ('wCentr', 'computeCentralised'),
                   ('wSSBC', 'computeSingleSensorBroadcast')):
        if case['danse'].get(fl, False):
            R = dv.nRounds
            errs = np.concatenate([_bin_rel(getattr(dv, wn)[k][:, 1:R + 1, :], getattr(ov, wn)[k][:, 1:R + 1, :]).ravel()
                                   for k in range(len(case['M']))])
            sw = _stats(errs)
            print('  ', wn, sw)
            assert sw['p99'] <= 1e-4, (wn, sw)
    # golden (reference itself): same d
    g = np.load(golden_dir / f"{case['name']}.npz")
    dg = rel_err(dv.d, g['d'])
    print('   d vs reference golden', dg)
    assert st['median'] <= 1e-5 and st['p99'] <= 1e-4, st
    assert de <= 1e-4
    assert dg <= 1e-4, dg


# Filter dimensions above 16 (64-lane solver class, solver64m.hpp): config C
# shape (K=16 x 4, D=19) and two ragged cases, compared with the float64
# oracle (the reference fixtures pin the oracle at smaller D); the same
# tolerance as every other class.
BIG_CASES = [
    dict(name='online_C_shape_K16_D19_asy', M=[4] * 16, dur=4.0, seed=21,
         danse=dict(ONLINE_CASES[1]['danse'], nodeUpdating='asy')),
    dict(name='online_big_D27_seq_r2', M=[24, 2, 3, 3], dur=4.0, seed=22,
         danse=dict(ONLINE_CASES[1]['danse'], nodeUpdating='seq', GEVDrank=2)),
    dict(name='online_big_D20_mwf', M=[17, 4, 4, 5], dur=4.0, seed=23,
         danse=dict(ONLINE_CASES[1]['danse'], nodeUpdating='asy', performGEVD=False)),
    # random filters + per-bin / per-node non-Hermitian SCM init on the 2D
    # classes (D = 15, centralised 24): the lower-triangle reading of eigh
    dict(name='online_big_init_random', M=[12, 6, 3, 3], dur=3.0, seed=24,
         danse=dict(next(c for c in ONLINE_CASES if c['name'] == 'online_init_random_asy')['danse'])),
    # the GEVD of classes 56 and 64 (D 49..64, update_kernel_big: row per
    # lane, runtime pivot loops) next to lane-class nodes
    dict(name='online_big_D51_asy', M=[48, 2, 2, 2], dur=6.0, seed=25,
         danse=dict(ONLINE_CASES[1]['danse'], nodeUpdating='asy')),
    dict(name='online_big_D60_seq_r2', M=[57, 2, 2, 2], dur=6.0, seed=26,
         danse=dict(ONLINE_CASES[1]['danse'], nodeUpdating='seq', GEVDrank=2)),
]


@pytest.mark.parametrize('case', BIG_CASES, ids=lambda c: c['name'])
def test_online_engine_large_D(case):
    from danse_amd.core import danse_multi
    from oracle import danse_ref_cpu as O
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    dv = danse_multi([sc], dp)[0]
    ov = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive)
    assert np.array_equal(dv.startRound, ov.startRound)
    assert np.array_equal(dv.nInternalFilterUps, ov.nInternalFilterUps)
    assert int(np.sum(dv.diag)) == 0
    st, de = _compare_online(case, dv, ov)
    assert st['median'] <= 1e-5 and st['p99'] <= 1e-4, st
    assert de <= 1e-4


@pytest.mark.parametrize('case', BATCH_CASES, ids=lambda c: c['name'])
def test_batch_engine_vs_oracle(case, golden_dir):
    """Device batch DANSE (MFMA Y.Y^H, STFT / ISTFT, MMSE cost) against the
    float64 oracle and the reference's own fixture."""
    from danse_amd.core import danse_batch
    from oracle import danse_ref_cpu as O
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    out, _ = danse_batch(sc, dp)
    ov = O.danse_batch(sc, dp, vadMinProp=wp.vadMinProportionActive)
    nb = case['danse']['maxBatchUpdates'] + 1
    errs = [_bin_rel(out.wTilde[k][:, 1:nb, :], ov.wTilde[k][:, 1:nb, :]).ravel() for k in range(len(case['M']))]
    st = _stats(np.concatenate(errs))
    de = rel_err(out.d, ov.d)
    ce = float(np.max(np.abs(out.mmseCost - np.array(ov.mmseCost, dtype=float)) / np.abs(np.array(ov.mmseCost, dtype=float))))
    g = np.load(golden_dir / f"{case['name']}.npz")
    dg = rel_err(out.d, g['d'])
    print(case['name'], 'w', st, 'd', de, 'cost', ce, 'd vs golden', dg)
    assert st['median'] <= 1e-5 and st['p99'] <= 1e-4, st
    assert de <= 1e-4 and ce <= 1e-4 and dg <= 1e-4
    # centralised / local batch estimates (obs = 2 / 1 engines)
    for fam in ('Centr', 'Local'):
        if f'd{fam}' not in g:
            continue
        sf = _stats(np.concatenate([_bin_rel(getattr(out, f'w{fam}')[k][:, 1, :], getattr(ov, f'w{fam}')[k][:, 1, :]).ravel()
                                    for k in range(len(case['M']))]))
        dfe = rel_err(getattr(out, f'd{fam}'), getattr(ov, f'd{fam}'))
        dfg = rel_err(getattr(out, f'd{fam}'), g[f'd{fam}'])
        cr = np.array(getattr(ov, f'mmseCost{fam}'))
        cfe = float(np.max(np.abs(np.array(getattr(out, f'mmseCost{fam}')) - cr) / np.abs(cr)))
        print('  ', fam, 'w', sf, 'd', dfe, 'd vs golden', dfg, 'cost', cfe)
        assert sf['median'] <= 1e-5 and sf['p99'] <= 1e-4, sf
        assert dfe <= 1e-4 and dfg <= 1e-4 and cfe <= 1e-4


@pytest.mark.parametrize('case', BESTPERF_CASES, ids=lambda c: c['name'])
def test_best_perf_vs_oracle(case, golden_dir):
    """get_best_perf (d_core.py:602-627) on the device batch engine
    (obs = centralised): filters, estimate and MMSE cost against the float64
    oracle, and the noise-only / speech-only replays with the recorded
    filters against the reference's fixture."""
    import copy
    from danse_amd import core
    from danse_amd.params import PreComputedFilters
    from oracle import danse_ref_cpu as O
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    bp = core.get_best_perf(sc, dp)
    ob = O.get_best_perf(sc, dp, vadMinProp=wp.vadMinProportionActive)
    g = np.load(golden_dir / f"{case['name']}.npz")
    st = _stats(np.concatenate([_bin_rel(bp.wCentr[k][:, 1, :], ob.wCentr[k][:, 1, :]).ravel()
                                for k in range(len(case['M']))]))
    de, dg = rel_err(bp.dCentr, ob.dCentr), rel_err(bp.dCentr, g['dCentr'])
    ce = float(np.max(np.abs(np.array(bp.mmseCostCentr) - g['mmseCostCentr']) / g['mmseCostCentr']))
    print(case['name'], 'w', st, 'd', de, 'd vs golden', dg, 'cost', ce)
    assert st['median'] <= 1e-5 and st['p99'] <= 1e-4, st
    assert de <= 1e-4 and dg <= 1e-4 and ce <= 1e-4
    pU = copy.deepcopy(dp)
    for purpose in ('noise-only', 'speech-only'):
        pU.preGivenFilters = PreComputedFilters(active=True, purpose=purpose)
        o = core.get_best_perf(sc, pU, wCentr=bp.wCentr)
        e = rel_err(o.dCentr, g[f'dCentr_{purpose[0]}'])
        print('  ', purpose, e)
        assert e <= 1e-4, (purpose, e)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('M', [[8] * 12, [8] * 32], ids=['sumM96', 'sumM256'])
def test_best_perf_wide_vs_oracle(M):
    """get_best_perf at sum(M) > 64 (config D's K = 32 x 8 gives sum(M) =
    256): the wide classes (csrc/wide.hpp: float64 HERK on MFMA, one
    workgroup per bin for Cholesky, congruence, tridiagonalisation,
    multisection and inverse iteration) against the float64 oracle, whose
    get_best_perf is pinned to the reference's fixtures at K = 3 / 4
    (bestperf_*; the wide KATs pin the filter update itself at D = 96 / 256)."""
    from danse_amd import core
    from oracle import danse_ref_cpu as O
    from golden_cases import BATTERY
    # the centralised VAD is active when any node's is (d_classes.py:905-911):
    # with 12-32 nodes and the default 0.5 s pauses fewer frames than sum(M)
    # are noise-only and Rnn is singular (the reference's eigh raises too), so
    # the desired source pauses 1.5 s: 198 of 312 / 317 of 500 frames noise-only
    case = dict(name=f'bestperf_wide_{sum(M)}', M=M, dur=10.01 if sum(M) <= 96 else 16.01, seed=62 + len(M),
                danse=dict(BATTERY, nodeUpdating='asy', simType='batch'))
    sc = make_case_scene(case, pauseDuration=1.5)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    bp = core.get_best_perf(sc, dp)
    O.set_workers(8)
    try:
        ob = O.get_best_perf(sc, dp, vadMinProp=wp.vadMinProportionActive)
    finally:
        O.set_workers(0)
    K = len(M)
    assert bp.wCentr[0].shape[-1] == sum(M)
    st = _stats(np.concatenate([_bin_rel(bp.wCentr[k][:, 1, :], ob.wCentr[k][:, 1, :]).ravel() for k in range(K)]))
    de = rel_err(bp.dCentr, ob.dCentr)
    cr = np.array(ob.mmseCostCentr, dtype=float)
    ce = float(np.max(np.abs(np.array(bp.mmseCostCentr) - cr) / np.abs(cr)))
    print(case['name'], 'w', st, 'd', de, 'cost', ce)
    assert st['median'] <= 1e-5 and st['p99'] <= 1e-4, st
    assert de <= 1e-4 and ce <= 1e-4


def test_batch_covmats_op():
    """danse_batch_covmats (MFMA HERK) on random observations vs numpy."""
    L, lib = _lib()
    rng = np.random.default_rng(5)
    for (B, Tf, D) in [(7, 37, 5), (600, 50, 11), (3, 21, 39)]:
        Y = rng.standard_normal((B, Tf, D)) + 1j * rng.standard_normal((B, Tf, D))
        vad = (rng.random(Tf) > 0.4).astype(np.uint8)
        yd, vd = _dev_cf(Y), torch.from_numpy(vad).cuda()
        ry = torch.empty((B, D, D, 2), dtype=torch.float32, device='cuda')
        rn = torch.empty_like(ry)
        L.check(lib.danse_batch_covmats(ctypes.c_void_p(yd.data_ptr()), B, Tf, D, ctypes.c_void_p(vd.data_ptr()),
                                        ctypes.c_void_p(ry.data_ptr()), ctypes.c_void_p(rn.data_ptr()), None))
        torch.cuda.synchronize()
        v = vad.astype(bool)
        refy = np.mean(np.einsum('btj,btl->btjl', Y[:, v], Y[:, v].conj()), axis=1)
        refn = np.mean(np.einsum('btj,btl->btjl', Y[:, ~v], Y[:, ~v].conj()), axis=1)
        gy = ry.cpu().numpy().view(np.complex64)[..., 0]
        gn = rn.cpu().numpy().view(np.complex64)[..., 0]
        assert rel_err(gy, refy) < 2e-6 and rel_err(gn, refn) < 2e-6, (B, Tf, D, rel_err(gy, refy), rel_err(gn, refn))


def test_dxcp_vs_oracle():
    """Device DXCP-PhaT (batched pairs) against the float64 oracle, itself
    pinned bit-exactly to the reference's DXCPPhaT: per-frame SRO within
    0.05 ppm and STO within 0.05 samples, all three golden cases in one batch."""
    import warnings
    from golden_cases import DXCP_CASES, dxcp_inputs
    from danse_amd.dxcp import DXCPPhaTBatch
    from oracle import dxcp_ref as D
    ins = [dxcp_inputs(c) for c in DXCP_CASES]
    n = min(len(a) for a, _ in ins) // 2048
    est = DXCPPhaTBatch(len(DXCP_CASES))
    got = np.zeros((n, len(DXCP_CASES), 2))
    for i in range(n):
        fr = np.stack([np.stack((a[i * 2048:(i + 1) * 2048], b[i * 2048:(i + 1) * 2048])) for a, b in ins])
        sro, sto = est.process_frames(fr)
        got[i, :, 0] = sro.cpu().numpy()
        got[i, :, 1] = sto.cpu().numpy()
    est.close()
    for c, (a, b) in zip(DXCP_CASES, ins):
        j = DXCP_CASES.index(c)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore', DeprecationWarning)
            sro_o, sto_o = D.run(a[:n * 2048], b[:n * 2048])
        es, et = np.max(np.abs(got[:, j, 0] - sro_o)), np.max(np.abs(got[:, j, 1] - sto_o))
        print(c['name'], 'max |dSRO| ppm', es, 'max |dSTO|', et, 'final', got[-1, j])
        assert es <= 0.05 and et <= 0.05, (c['name'], es, et)


def test_tz_few_samples_vs_reference_fixtures():
    """T(z) few-samples compression through the reference-shaped drop-ins
    (danse_amd.tz.dist_fct_approx / danse_compression_few_samples) against the
    reference's own outputs (tz_* fixtures): relative error <= 1e-5 on the
    IR and on the broadcast samples."""
    from golden_cases import TZ_CASES, tz_inputs
    from danse_amd import tz
    from pathlib import Path
    gdir = Path(__file__).resolve().parent / 'golden'
    for c in TZ_CASES:
        g = dict(np.load(gdir / f"{c['name']}.npz", allow_pickle=False))
        wHat, yq, h, f, wPrev = tz_inputs(c)
        z, wIR = tz.danse_compression_few_samples(yq, wHat, c['L'], wPrev, h, f, c['Ns'],
                                                  updateBroadcastFilter=c['update'])
        ew, ez = rel_err(wIR, g['wIR']), rel_err(z, g['z'])
        print(c['name'], 'wIR', ew, 'z', ez)
        assert ew < 1e-5 and ez < 1e-5, (c['name'], ew, ez)


@pytest.mark.parametrize('M,L', [(1, 1), (2, 7), (3, 100), (4, 512), (5, 1024), (9, 333)])
def test_tz_batched_vs_oracle(M, L):
    """B = 37 nodes per launch (TZCompressor) against the float64 oracle
    (closed-form IR, itself pinned to the reference's dist_fct_approx), ragged
    L (not a multiple of the 8-output tile) and M above the 4-sensor LDS pass."""
    from danse_amd.tz import TZCompressor
    from oracle import tz_ref as T
    rng = np.random.default_rng(1000 + 10 * M + L)
    N, B = 1024, 37
    h = np.sqrt(np.hanning(N))
    f = rng.uniform(0.2, 1.0, N)
    wHat = rng.standard_normal((B, N // 2 + 1, M)) + 1j * rng.standard_normal((B, N // 2 + 1, M))
    yq = rng.standard_normal((B, N, M))
    c = TZCompressor(h, f, 512)
    wIR = c.ir(wHat)
    z = c.compress(yq, wIR, L).cpu().numpy()
    wIRh = wIR.cpu().numpy()
    c.close()
    for b in range(B):
        ref_ir = T.dist_fct_approx_closed(wHat[b], h.astype(np.float32).astype(np.float64),
                                          f.astype(np.float32).astype(np.float64), 512)
        assert rel_err(wIRh[b], ref_ir) < 1e-5, (b, rel_err(wIRh[b], ref_ir))
        # the convolution on the device's own IR: isolates the compress kernel
        zr = np.zeros(L)
        for m in range(M):
            zr += T.extract_few_samples_from_convolution(np.arange(2 * N - 1 - L + 1, 2 * N), wIRh[b, :, m].astype(np.float64),
                                                         yq[b, :, m].astype(np.float32).astype(np.float64))
        assert rel_err(z[b], zr) < 1e-5, (b, rel_err(z[b], zr))


def test_batched_scenes_are_independent():
    """S scenes in one engine give the same results as one scene alone."""
    from danse_amd.core import danse_multi
    case = ONLINE_CASES[1]
    dp, wp = make_case_params(case)
    scenes = []
    for seed in (11, 12, 13):
        sc = make_case_scene(dict(case, seed=seed))
        sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
        scenes.append(sc)
    multi = danse_multi(scenes, dp)
    for s, sc in enumerate(scenes):
        one = danse_multi([sc], dp)[0]
        assert np.array_equal(one.d, multi[s].d)
        for k in range(len(case['M'])):
            assert np.array_equal(one.wTilde[k], multi[s].wTilde[k])


def test_snr_replay_vs_oracle():
    """Pre-given filter replay (generate_signals_for_snr_computation)."""
    from danse_amd import core
    from oracle import danse_ref_cpu as O
    case = ONLINE_CASES[0]
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    ov = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive)
    sig_o = O.generate_signals_for_snr_computation(sc, dp, ov, vadMinProp=wp.vadMinProportionActive)
    # replay the ORACLE's filters on the device: isolates the replay path
    sig_g = core.generate_signals_for_snr_computation(dp, ov, sc)
    for key in ('n', 's'):
        e = rel_err(sig_g[key], sig_o[key])
        print('replay', key, e)
        assert e < 1e-5


@pytest.mark.parametrize('case', BATCH_CASES, ids=lambda c: c['name'])
def test_batch_node_sharded_equals_full(case):
    """Node-sharded batch DANSE (two engines of one device, each owning a
    node block, exchanging the external filters after every iteration as
    the RCCL all-gather would) against the single-engine run: every owned
    node's filters, estimates and costs, and every node's external filters,
    agree (same kernels on the same bins: bit-exact expected, 1e-6 tested)."""
    import torch
    from danse_amd.batch import BatchEngine, node_ranges
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    dp.simType = 'batch'
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    full = BatchEngine([sc], dp).run().outputs()[0]
    K = len(case['M'])
    rngs, c = node_ranges(K, 2)
    engs = [BatchEngine([sc], dp, nodeRange=r) for r in rngs]
    bufs = [torch.zeros(c * e.S * e.wext_chunk(), dtype=torch.complex64, device='cuda:0') for e in engs]
    for it in range(engs[0].iters):
        for e, b in zip(engs, bufs):
            e.run_iters(it, it + 1)
            e.pack_wext(it + 1, b)
        g = torch.cat(bufs)
        for e in engs:
            e.unpack_wext(it + 1, g)
    torch.cuda.synchronize()
    exact = True
    for e, (k0, k1) in zip(engs, rngs):
        o = e.outputs()[0]
        for k in range(K):
            exact &= np.array_equal(o.wTildeExt[k], full.wTildeExt[k])
            assert np.allclose(o.wTildeExt[k], full.wTildeExt[k], rtol=1e-6, atol=1e-7), (k0, k)
        for k in range(k0, k1):
            for a, b in ((o.wTilde[k], full.wTilde[k]), (o.d[:, k], full.d[:, k]), (o.dhat[:, :, k], full.dhat[:, :, k]),
                         (o.mmseCost[:, k], full.mmseCost[:, k])):
                exact &= np.array_equal(a, b)
                assert np.allclose(a, b, rtol=1e-6, atol=1e-7), (k0, k)
        for k in set(range(K)) - set(range(k0, k1)):
            # not this engine's outputs: marked, never leftover device memory
            assert o.wTilde[k] is None
            assert np.isnan(o.d[:, k]).all() and np.isnan(o.mmseCost[:, k]).all()
        e.close()
    print(case['name'], 'bit-exact' if exact else 'within 1e-6')


@pytest.mark.timeout(600)
def test_batch_engine_config_D_shape_vs_oracle():
    """Config D's shape end to end through BatchEngine: K = 32 nodes x 8 mics
    (D = 39: the 256-channel STFT, z of 32 senders, the HERK padded 39 -> 48,
    the 2D solver class, ISTFT and MMSE cost), asy, T = 10.01 s, against the
    float64 oracle (pinned to the reference's batch fixtures at K = 3) for
    two batch iterations (the oracle's per-bin eigh costs ~11 s per
    iteration at D = 39)."""
    from danse_amd.core import danse_batch
    from oracle import danse_ref_cpu as O
    from golden_cases import BATTERY
    case = dict(name='batch_D_K32x8_asy', M=[8] * 32, dur=10.01, seed=61,
                danse=dict(BATTERY, nodeUpdating='asy', simType='batch', maxBatchUpdates=2))
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    out, _ = danse_batch(sc, dp)
    ov = O.danse_batch(sc, dp, vadMinProp=wp.vadMinProportionActive)
    K = 32
    errs = [_bin_rel(out.wTilde[k][:, 1:3, :], ov.wTilde[k][:, 1:3, :]).ravel() for k in range(K)]
    st = _stats(np.concatenate(errs))
    de = rel_err(out.d, ov.d)
    dhe = rel_err(out.dhat, ov.dhat)
    cr = np.array(ov.mmseCost, dtype=float)
    ce = float(np.max(np.abs(out.mmseCost - cr) / np.abs(cr)))
    print(case['name'], 'w', st, 'd', de, 'dhat', dhe, 'cost', ce)
    assert out.wTilde[0].shape[-1] == 39
    assert st['median'] <= 1e-5 and st['p99'] <= 1e-4, st
    assert de <= 1e-4 and dhe <= 1e-4 and ce <= 1e-4
