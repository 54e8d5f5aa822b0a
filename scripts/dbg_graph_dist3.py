"""Debug: does a non-captured RCCL collective between replays of a CUDA graph
that contains RCCL all-gathers break the later replays (world size 1)?
Variants: the out-of-graph all_reduce on the same communicator, on a second
NCCL group, on a gloo group."""
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
os.environ.setdefault('MASTER_PORT', '29735')
torch.cuda.set_device(0)
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda:0'))
g_nccl2 = dist.new_group([0], backend='nccl')
g_gloo = dist.new_group([0], backend='gloo')

from test_gpu_dist import CASES, _setup  # noqa: E402
from danse_amd.dist import ShardedRun, ShardedEngine  # noqa: E402
from danse_amd.engine import DanseEngine  # noqa: E402
from danse_amd import _lib as L  # noqa: E402

sc, dp, wp = _setup(CASES['plain_k4'])


def grab(e):
    torch.cuda.synchronize()
    return e._get(L.OUT_D, 0, dtype=np.float32).copy(), e._get(L.OUT_W, 0, 0).copy()


def same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


for mode in ('same-comm', 'second-nccl', 'gloo', 'none'):
    eng = DanseEngine([sc], dp)
    run = ShardedRun(ShardedEngine(eng), graph=False)
    eng.begin_run(speculative=False)
    run._rounds(True, False)
    ref = grab(eng)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        run._rounds(True, False)
    res = []
    for i in range(4):
        g.replay()
        res.append(same(grab(eng), ref))
        if mode == 'same-comm':
            t = torch.ones(1, device='cuda:0')
            dist.all_reduce(t)
        elif mode == 'second-nccl':
            t = torch.ones(1, device='cuda:0')
            dist.all_reduce(t, group=g_nccl2)
        elif mode == 'gloo':
            t = torch.ones(1)
            dist.all_reduce(t, group=g_gloo)
        torch.cuda.synchronize()
    print(mode, 'replays equal to eager:', res, flush=True)
    eng.close()
dist.destroy_process_group()
