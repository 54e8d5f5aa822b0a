"""Debug: torch CUDA-graph capture of the sharded round sequence (world 1,
RCCL) -- which replays differ from the eager run, and where."""
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
os.environ.setdefault('MASTER_PORT', '29731')
torch.cuda.set_device(0)
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda:0'))

from test_gpu_dist import CASES, _setup  # noqa: E402
from danse_amd.dist import ShardedRun, ShardedEngine  # noqa: E402
from danse_amd.engine import DanseEngine  # noqa: E402
from danse_amd import _lib as L  # noqa: E402

sc, dp, wp = _setup(CASES['plain_k4'])


def grab(e):
    torch.cuda.synchronize()
    return e._get(L.OUT_D, 0, dtype=np.float32).copy(), e._get(L.OUT_W, 0, 0).copy(), e._get(L.OUT_DHAT, 0).copy()


def report(tag, a, b):
    for nm, x, y in zip(('d', 'w0', 'dhat'), a, b):
        if np.array_equal(x, y):
            print(f'{tag} {nm}: equal')
        else:
            i = int(np.flatnonzero(x != y)[0])
            print(f'{tag} {nm}: DIFF first index {i} of {x.size}, max abs {float(np.max(np.abs(x - y))):.3e}')


for mode in ('exchange', 'noexchange', 'nogate'):
    eng = DanseEngine([sc], dp)
    run = ShardedRun(ShardedEngine(eng))
    if mode == 'noexchange':
        run.exchange = lambda r=0: None
    gate = mode != 'nogate'
    eng.begin_run(speculative=gate)
    run._rounds(True, gate)
    ref = grab(eng)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        run._rounds(True, gate)
    for i in range(3):
        g.replay()
        report(f'{mode} replay {i}', grab(eng), ref)
    # eager again after the replays
    run._rounds(True, gate)
    report(f'{mode} eager-after', grab(eng), ref)
    eng.close()
# the engine's own hipGraph for comparison
eng = DanseEngine([sc], dp)
eng.run(graph=False)
ref = grab(eng)
for i in range(3):
    L.check(eng.lib.danse_engine_reset(eng.eng, eng.stream_ptr()), eng.eng)
    eng.run(graph=True)
    report(f'hipgraph run {i}', grab(eng), ref)
dist.destroy_process_group()
