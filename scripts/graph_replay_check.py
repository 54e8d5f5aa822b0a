"""GPU check, one process, no torch.distributed: does a CUDA graph of the
online rounds replay bit-equal to the eager run, with and without the state
reset (hipMemsetAsync nodes + reset kernels) and the speculative gate (its
0xff verdict memset) inside the graph, and with the engine's host-side
bookkeeping (begin_run) between replays?

Also a micro check of raw memset nodes: hipMemsetAsync (through ctypes on
libamdhip64) + an in-place torch add captured into one graph, replayed 4x.

Prints one line per variant: the per-replay equality with the eager run and
the largest |d| difference.  Used to settle the cause of the round-3 pass-2
mismatch of test_rccl_graph_captured_rounds."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / 'tests', ROOT / 'tests' / 'golden'):
    sys.path.insert(0, str(p))

from test_gpu_dist import CASES, _setup  # noqa: E402
from danse_amd.dist import ShardedEngine  # noqa: E402
from danse_amd.engine import DanseEngine  # noqa: E402
from danse_amd import _lib as L  # noqa: E402

torch.cuda.set_device(0)


def grab(e):
    torch.cuda.synchronize()
    return [e._get(L.OUT_D, 0, dtype=np.float32).copy()] + [e._get(L.OUT_W, 0, k).copy() for k in range(e.K)]


def maxdiff(a, b):
    return max(float(np.max(np.abs(x - y))) for x, y in zip(a, b))


def memset_micro():
    """Raw memset nodes: hipMemsetAsync (ctypes, libamdhip64) of a zero fill
    and of a 0xff fill, each followed by an in-place torch add, captured into
    one graph and replayed 4x; reported per buffer.  Then the same with the
    engine's fill kernel (danse_mi355x_fill, csrc/fill.hpp) in place of the
    memsets."""
    hip = ctypes.CDLL('libamdhip64.so')
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    hip.hipMemsetAsync.restype = ctypes.c_int
    lib = L.load_library()
    for how in ('hipMemsetAsync', 'fill kernel'):
        res = []
        for n in (16, 4096, 1 << 22):
            a = torch.zeros(n // 4, dtype=torch.int32, device='cuda:0')
            b = torch.zeros(n // 4, dtype=torch.int32, device='cuda:0')
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.graph(g, stream=side):
                st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                if how == 'hipMemsetAsync':
                    assert hip.hipMemsetAsync(ctypes.c_void_p(a.data_ptr()), 0, n, st) == 0
                    assert hip.hipMemsetAsync(ctypes.c_void_p(b.data_ptr()), 0xff, n, st) == 0
                else:
                    assert lib.danse_mi355x_fill(ctypes.c_void_p(a.data_ptr()), 0, n, st) == 0
                    assert lib.danse_mi355x_fill(ctypes.c_void_p(b.data_ptr()), 0xff, n, st) == 0
                a.add_(1)
                b.add_(1)
            oka, okb = [], []
            for _ in range(4):
                g.replay()
                torch.cuda.synchronize()
                oka.append(int(a[0].item()) if not bool(torch.all(a == 1)) else 'ok')
                okb.append(int(b[0].item()) if not bool(torch.all(b == 0)) else 'ok')
            res.append((n, 'zero fill', oka, '0xff fill', okb))
        print(f'{how} in a graph (bytes, per replay ok or the value found):', res, flush=True)


def variant(name, reset_in, gate, host_between):
    sc, dp, wp = _setup(CASES['plain_k4'])
    eng = DanseEngine([sc], dp)
    se = ShardedEngine(eng)
    eng.run(graph=False)
    ref = grab(eng)

    def rounds(reset):
        if reset:
            se.reset()
        for r in range(eng.R):
            se.bcast(r)
            if gate:
                se.gate_launch(r)
            se.update(r)
        se.finish()

    eng.begin_run(speculative=gate)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        rounds(reset_in)
    ok, diffs, gok = [], [], []
    for i in range(3):
        if host_between and i > 0:
            eng.begin_run(speculative=gate)
        if not reset_in:
            se.reset()
        g.replay()
        out = grab(eng)
        ok.append(all(np.array_equal(x, y) for x, y in zip(out, ref)))
        diffs.append(maxdiff(out, ref))
        if gate:
            gok.append(eng.gate_ok())
    print(f'{name:34s} replays equal to eager: {ok} max|diff| {["%.2e" % d for d in diffs]}'
          f' gate verdicts ok: {gok}', flush=True)
    eng.close()


memset_micro()
for reset_in in (True, False):
    for gate in (False, True):
        for hb in (False, True):
            variant(f'reset_in={int(reset_in)} gate={int(gate)} begin_run={int(hb)}', reset_in, gate, hb)
