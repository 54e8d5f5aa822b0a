"""Shared helpers for the tests (case -> params/scene)."""
from __future__ import annotations

import numpy as np

from danse_amd import params as P
from danse_amd.scene import make_scene


def make_case_params(case, SROperNode=None):
    if SROperNode is None:
        SROperNode = case.get('sros')
    kw = dict(case['danse'])
    if isinstance(kw.get('cohDrift'), dict):
        kw['cohDrift'] = P.CohDriftParameters(**kw['cohDrift'])
    dp = P.DANSEparameters(**kw)
    wp = P.WASNparameters(trueRoom=False, signalType='random', nSensorPerNode=list(case['M']),
                          SROperNode=np.zeros(len(case['M'])) if SROperNode is None else np.asarray(SROperNode),
                          topologyParams=P.TopologyParameters(topologyType='fully-connected', seed=12348))
    wp.__post_init__()
    dp.__post_init__()
    dp.get_wasn_info(wp)
    return dp, wp


def make_case_scene(case, **kw):
    if 'sros' in case and 'SROperNode' not in kw:
        kw['SROperNode'] = case['sros']
    return make_scene(case['M'], sigDur=case['dur'], seed=case.get('seed', 0), **kw)


def rel_err(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    if b.size == 0:
        return 0.0
    den = np.max(np.abs(b))
    return float(np.max(np.abs(a - b)) / (den if den > 0 else 1.0))
