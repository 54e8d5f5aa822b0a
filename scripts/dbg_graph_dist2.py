"""Debug: the exact flow of tests/test_gpu_dist.py::test_rccl_graph_captured_rounds
(world 1, RCCL): per pass, which outputs differ from the single-engine run,
whether the speculative gate failed, and the verdicts."""
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / 'tests', ROOT / 'tests' / 'golden'):
    sys.path.insert(0, str(p))
os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
os.environ.setdefault('MASTER_PORT', '29733')
torch.cuda.set_device(0)
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda:0'))

from test_gpu_dist import CASES, _setup  # noqa: E402
from danse_amd.dist import ShardedRun, ShardedEngine  # noqa: E402
from danse_amd.engine import DanseEngine  # noqa: E402
from danse_amd.core import danse_multi  # noqa: E402

sc, dp, wp = _setup(CASES['plain_k4'])
ref = danse_multi([sc], dp)[0]
eng = DanseEngine([sc], dp)
run = ShardedRun(ShardedEngine(eng))
orig_ok = eng.gate_ok


def ok_spy(stream=None):
    v = orig_ok(stream)
    print('   gate_ok ->', v, flush=True)
    return v


eng.gate_ok = ok_spy
for i in range(5):
    skip_outputs = i >= 3
    run.run(reset=True)
    torch.cuda.synchronize()
    print(f'pass {i}: graphs {len(run._graphs)} specfail {eng.gate_spec_failed}', flush=True)
    o = eng.outputs()[0]
    for k in range(4):
        for nm, a, b in (('d', o.d[:, k], ref.d[:, k]), ('w', o.wTilde[k], ref.wTilde[k]),
                         ('e', o.wTildeExt[k], ref.wTildeExt[k])):
            if not np.array_equal(a, b):
                idx = np.argwhere(a != b)[0]
                print(f'   node {k} {nm} DIFF at {idx.tolist()} max {float(np.max(np.abs(a - b))):.3e}', flush=True)
dist.destroy_process_group()
