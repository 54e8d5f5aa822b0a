"""CPU-side checks of the drop-in boundary: the C-ABI library builds/loads and
exports every symbol include/danse_mi355x.h declares (no compute calls — no
GPU here), the ctypes struct matches the header, and the host schedule tables."""
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _header_functions():
    txt = (ROOT / 'include' / 'danse_mi355x.h').read_text()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(danse_[a-z_0-9]+)\s*\(', txt)))


def test_library_exports_every_header_symbol():
    from danse_amd import _lib as L
    from danse_amd import build as B
    B.build(verbose=False)
    lib = L.load_library()
    names = _header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
        assert n in L.SIGNATURES, f'{n} missing from the ctypes signatures'


def test_cfg_struct_matches_header_fields():
    from danse_amd import _lib as L
    txt = (ROOT / 'include' / 'danse_mi355x.h').read_text()
    body = txt[txt.index('typedef struct danse_cfg {') + len('typedef struct danse_cfg {'):txt.index('} danse_cfg;')]
    body = re.sub(r'/\*.*?\*/', '', body, flags=re.S)
    fields = []
    for decl in body.split(';'):
        decl = decl.strip()
        if not decl or decl.startswith('typedef'):
            continue
        fields += [x.strip().lstrip('*') for x in re.sub(r'^(const\s+)?\w+\**\s+', '', decl).split(',')]
    assert [f for f, _ in L.DanseCfg._fields_] == fields


def test_product_has_no_oracle_dependency():
    """The product package must never import the oracle (test infrastructure)."""
    for p in (ROOT / 'danse_amd').rglob('*.py'):
        src = p.read_text()
        assert 'import oracle' not in src and 'from oracle' not in src, p


def test_round_tables_sync_schedule():
    from danse_amd.scene import make_scene
    from danse_amd.scheduler import initialize_events, compile_rounds
    from _util import make_case_params
    case = dict(M=[2, 2, 2], danse=dict(simType='online', nodeUpdating='seq'))
    dp, wp = make_case_params(case)
    sc = make_scene([2, 2, 2], sigDur=2.0, seed=0)
    ev, fs = initialize_events([n.timeStamps for n in sc.wasn], [n.fs for n in sc.wasn], dp,
                               [n.neighborsIdx for n in sc.wasn])
    rt = compile_rounds(ev, fs, dp, 3)
    T = 32000
    assert rt.nRounds == (T - 1) // 512 - 2
    j = np.arange(2, 2 + rt.nRounds)
    assert np.array_equal(rt.bcEnd[:, 0], j * 512)
    assert np.array_equal(rt.upEnd[:, 0], j * 512 - 512)
    # seq: exactly one updating node per round, round robin
    assert np.array_equal(rt.doSolve.sum(axis=1), np.ones(rt.nRounds))
    assert np.array_equal(np.argmax(rt.doSolve, axis=1), np.arange(rt.nRounds) % 3)


def test_round_tables_sro_schedule():
    """SRO clocks (quirk Q13): node 2 (fastest) updates before node 1 before
    node 0 at every round, so a faster receiver consumes a slower sender's
    frame of the previous round (lag 1); the first update sees an empty
    buffer (flag -N) from a lagging sender and Ns of N samples otherwise
    (flag -Ns, quirk Q5); later buffers hold exactly Ns (flag 0)."""
    from danse_amd.scene import make_scene
    from danse_amd.scheduler import initialize_events, compile_rounds
    from _util import make_case_params
    case = dict(M=[1, 1, 1], danse=dict(simType='online', nodeUpdating='asy'))
    dp, wp = make_case_params(case, SROperNode=[0, 100, 200])
    sc = make_scene([1, 1, 1], sigDur=2.0, seed=0, SROperNode=[0, 100, 200])
    ev, fs = initialize_events([n.timeStamps for n in sc.wasn], [n.fs for n in sc.wasn], dp,
                               [n.neighborsIdx for n in sc.wasn])
    rt = compile_rounds(ev, fs, dp, 3)
    assert not rt.synchronous
    lag = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0]])
    assert all(np.array_equal(rt.zLag[r], lag) for r in range(rt.nRounds))
    assert np.array_equal(rt.flags[0], np.array([[0, -512, -512], [-1024, 0, -512], [-1024, -1024, 0]]))
    assert not np.any(rt.flags[1:])
    # frame ends: floor(t * fs_k) on each node's own clock (quirk Q3)
    assert np.all(np.abs(rt.bcEnd - (np.arange(2, 2 + rt.nRounds) * 512)[:, None]) <= 1)
    assert np.array_equal(rt.upEnd, rt.bcEnd - 512)


def test_compile_rounds_rejects_few_samples():
    """The wholeChunk compiler refuses fewSamples; compile_rounds_fs takes it."""
    from danse_amd.scene import make_scene
    from danse_amd.scheduler import initialize_events, compile_rounds
    from _util import make_case_params
    case = dict(M=[1, 1], danse=dict(simType='online', nodeUpdating='seq', broadcastType='fewSamples',
                                     broadcastLength=8))
    dp, wp = make_case_params(case)
    sc = make_scene([1, 1], sigDur=1.0, seed=0)
    ev, fs = initialize_events([n.timeStamps for n in sc.wasn], [n.fs for n in sc.wasn], dp,
                               [n.neighborsIdx for n in sc.wasn])
    with pytest.raises(NotImplementedError):
        compile_rounds(ev, fs, dp, 2)


@pytest.mark.parametrize('sros', [None, [0, 200]])
def test_round_tables_few_samples(sros):
    """fewSamples + efficientSpSBC (config E shape): the first broadcast sends
    L floor(N / L) samples, later ones Ns; streams are append-only (POS is
    the running sum of LEN); each round's z frame ends at the sender's stream
    length; the T(z) IR is refreshed from the node's current wExt iteration
    once per upTDfilterEvery = 1 s, never at single-sensor nodes."""
    from danse_amd.scene import make_scene
    from danse_amd.scheduler import initialize_events, compile_rounds_fs, FS_BCEND, FS_LEN, FS_POS, FS_IRSRC, FS_ZEND
    from _util import make_case_params
    M = [2, 3] if sros else [2, 3, 1]
    case = dict(M=M, danse=dict(simType='online', nodeUpdating='asy', broadcastType='fewSamples',
                                broadcastLength=128, noFusionAtSingleSensorNodes=True))
    kw = dict(SROperNode=sros) if sros else {}
    dp, wp = make_case_params(case, **kw)
    sc = make_scene(M, sigDur=2.5, seed=0, **kw)
    ev, fs = initialize_events([n.timeStamps for n in sc.wasn], [n.fs for n in sc.wasn], dp,
                               [n.neighborsIdx for n in sc.wasn])
    rt = compile_rounds_fs(ev, fs, dp, len(M), [n.timeStamps for n in sc.wasn], M)
    t = rt.fsTab
    assert rt.synchronous == (sros is None)
    for k in range(len(M)):
        assert np.array_equal(t[1:, k, FS_POS], np.cumsum(t[:-1, k, FS_LEN]))
        assert np.all(t[1:, k, FS_LEN] == 512)
        assert np.all(t[:, k, FS_ZEND] == t[:, k, FS_POS] + t[:, k, FS_LEN])
        src = t[:, k, FS_IRSRC]
        rr = np.nonzero(src >= 0)[0]
        assert np.array_equal(src[rr], rr)
        assert len(rr) == (0 if M[k] == 1 else 2)
    if sros is None:
        assert np.all(t[0, :, FS_LEN] == 1024) and not np.any(rt.flags)
        assert np.array_equal(t[:, :, FS_BCEND], rt.upEnd)
    else:
        # node 0 (slow clock) broadcasts at node 1's earlier update instant,
        # snapped to its own 128-sample grid: 896 samples, flag -128 at node 1
        assert t[0, 0, FS_LEN] == 896 and rt.flags[0, 1, 0] == -128
    assert np.array_equal(rt.bcEnd[:-1], rt.upEnd[1:])


def test_yaml_config_loads():
    from danse_amd.params import TestParameters
    p = TestParameters().load_from_yaml(str(ROOT / 'config_files' / 'sandbox_config_offline.yaml'))
    assert p.is_fully_connected_wasn()
    assert p.danseParams.Ns == 512 and p.danseParams.performGEVD
    assert list(p.wasnParams.nSensorPerNode) == [1, 1]


def test_get_metrics_rejects_metrics_off_the_device_path():
    """PESQ / SI-SNR, dynamic metrics and bestPerfData raise before any
    device work (danse_amd/metrics.py get_metrics; snr, fwSNRseg and
    (e)STOI are on the device)."""
    import numpy as np
    import pytest
    from danse_amd import metrics as DM
    x = np.zeros(4000)
    for m in (['pesq'], ['snr', 'sisnr'], ['stoi', 'pesq']):
        with pytest.raises(NotImplementedError):
            DM.get_metrics(x, x, x, x, x, metricsToPlot=m)
    with pytest.raises(NotImplementedError):
        DM.get_metrics(x, x, x, x, x, metricsToPlot=['snr'], dynamic=object())


def test_library_build_id_matches_sources():
    """The shipped library is the build of the shipped sources: build.py
    embeds the sources' hash, _lib refuses a mismatch."""
    from danse_amd import build as B
    from danse_amd import _lib as L
    lib = L.load_library()
    assert lib.danse_mi355x_build_id().decode() == B.source_hash()
    assert B.embedded_hash(L.LIB_PATH) == B.source_hash()
