"""Debug: online engine vs oracle for the init variants separately (GPU)."""
import sys
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'tests/golden')
from _util import make_case_scene, make_case_params, rel_err
from golden_cases import ONLINE_CASES
from danse_amd.core import danse_multi
from oracle import danse_ref_cpu as O
base = next(c for c in ONLINE_CASES if c['name'] == 'online_init_random_asy')
for label, mod in [('random_w_only', dict(covMatSameInitForAllFreqs=True, covMatSameInitForAllNodes=True)),
                   ('perbin_only', dict(filterInitType='selectFirstSensor')),
                   ('pernode_only', dict(filterInitType='selectFirstSensor', covMatSameInitForAllFreqs=True)),
                   ('both', {})]:
    case = dict(base, danse=dict(base['danse'], **mod))
    sc = make_case_scene(case)
    dp, wp = make_case_params(case)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    dv = danse_multi([sc], dp)[0]
    ov = O.danse(sc, dp, vadMinProp=wp.vadMinProportionActive)
    print(label, 'start', dv.startRound, ov.startRound, 'd', rel_err(dv.d, ov.d), 'dLocal', rel_err(dv.dLocal, ov.dLocal),
          'dCentr', rel_err(dv.dCentr, ov.dCentr), flush=True)
