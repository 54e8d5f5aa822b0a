"""Debug: DXCP-in-the-loop device run vs the oracle fed the same estimates,
and the same scene in Oracle mode (device vs oracle), to isolate the
DXCP-specific difference."""
import sys
import numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, 'tests/golden'); sys.path.insert(0, '.')
from danse_amd.core import danse_multi
from danse_amd.scene import make_scenes_device
from oracle import danse_ref_cpu as O
from _util import make_case_params
from golden_cases import BATTERY, _d

sros = [0.0, 120.0, -80.0]
M = [2, 2, 2]
K = 3
for mode in ('Oracle', 'DXCPPhaT'):
    case = dict(M=M, sros=sros, danse=_d(BATTERY, nodeUpdating='asy', compensateSROs=True, includeFSDflags=True,
                                         estimateSROs=mode))
    dp, wp = make_case_params(case)
    scenes, _ = make_scenes_device(M, 1, sigDur=12.0, seed=3, SROperNode=sros, host_signals=True)
    sc = scenes[0]
    for nd in sc.wasn:
        for f in ('data', 'cleanspeech', 'cleannoise'):
            setattr(nd, f, getattr(nd, f).astype(np.float64))
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    dv = danse_multi([sc], dp)[0]
    R = dv.nRounds
    kw = {}
    if mode == 'DXCPPhaT':
        kw['sroEstimates'] = [dv.SROsResiduals[k] for k in range(K)]
    ov = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive, **kw)
    print(mode, 'R', R, 'start dev', dv.startRound, 'oracle', ov.startRound, 'ups dev', dv.nInternalFilterUps,
          'oracle', ov.nInternalFilterUps, flush=True)
    for k in range(K):
        wg, wr = dv.wTilde[k][:, 1:R + 1, :], ov.wTilde[k][:, 1:R + 1, :]
        e = np.linalg.norm(wg - wr, axis=-1) / np.maximum(np.linalg.norm(wr, axis=-1), 1e-30)   # [F][R]
        med = np.median(e, axis=0)
        first = int(np.argmax(med > 1e-3)) if np.any(med > 1e-3) else -1
        print(' node', k, 'median err per round (every 20th):', np.array2string(med[::20], precision=2),
              'first round > 1e-3:', first, flush=True)
        if mode == 'DXCPPhaT':
            print('   residual rows 0..12:', np.array2string(dv.SROsResiduals[k][:12, 0] * 1e6, precision=2))
