"""Per-wave phase clocks of one round's update_kernel_2d launch (diagnostics).

Needs the 'stamp' build of the library (danse_amd.build variant: the kernel
records s_memtime marks at its phase boundaries):

    DANSE_LIB=danse_amd/libdanse_stamp.so DANSE_UPDATE_TRACE=250 \\
        python scripts/update_trace.py --workload N2

Marks (kernels_2d.hpp stamp(i)): 0 start, 1 y staged, 2 Rnn block loaded /
recursed / stored, 3 factor (rank-one record move or full factorisation,
factor-cache store) or cached factor loaded, 4 Ryy block loaded / recursed /
stored, 5 congruence, 6 solve (Lanczos or Householder path), 7 tail issued,
8 tail stores drained.  Path code bits: 1 noise frame (Rnn updated), 2 rank-one
factor move, 4 full factorisation, 8 cached factor reused, 16 solve, 32 / 64
warm Lanczos accepted / sent back.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

PHASES = ['y', 'Rnn', 'factor', 'Ryy', 'congr', 'solve', 'tail', 'drain']
# update_kernel_lane (D <= 12): 1 observation loaded, 2 Rnn recursion (noise
# frames), 3 factor (float64 Cholesky + inverse, or the cached factor into
# LDS), 4 Ryy recursion, 5 congruence, 6 eigen part + filter, 7 / 8 as above
PHASES_LANE = ['y', 'Rnn', 'factor', 'Ryy', 'congr', 'eigen', 'tail', 'drain']
# update_kernel_2dc (code bit 128; 256 = the noise-frame variant): 1 y staged,
# 2 C upper blocks (VAD) / factor moved + cached (noise), 3 C loaded (noise),
# 4 C moved + stored, 5 Lanczos, 6 w, 7 tail issued, 8 recursion + drain
PHASES_LEAN = ['y', 'Cfill/factor', 'Cload', 'Cmove', 'lanczos', 'w', 'tail', 'rec+drain']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='N2')
    ap.add_argument('--scenes', type=int, default=None)
    args = ap.parse_args()
    import bench
    import torch
    from danse_amd.engine import DanseEngine
    from danse_amd.scene import make_scene
    r = int(os.environ['DANSE_UPDATE_TRACE'])
    wl = bench.WORKLOADS[args.workload]
    S = args.scenes or wl.get('scenes', 1)
    dp, wp = bench._wl_params(wl)
    scenes = []
    for sd in range(S):
        sc = make_scene(wl['M'], sigDur=wl['dur'], seed=1000 + sd, SROperNode=wl.get('sros'))
        sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
        scenes.append(sc)
    eng = DanseEngine(scenes, dp)
    for _ in range(3):
        eng.run()
    torch.cuda.synchronize()
    n = ctypes.c_size_t(0)
    eng.lib.danse_engine_resident_trace(eng.eng, None, ctypes.byref(n))
    buf = np.zeros(n.value // 8, dtype=np.uint64)
    eng.lib.danse_engine_resident_trace(eng.eng, buf.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n))
    eng.close()
    t = buf.reshape(-1, 10)
    t = t[(t[:, 0] != 0) & np.all(t[:, :9] != 0, axis=1)]
    phases = PHASES_LANE if max(wl['M']) + len(wl['M']) - 1 <= 12 else PHASES
    marks, code = t[:, :9].astype(np.int64), t[:, 9]
    dt = np.diff(marks, axis=1)
    life = marks[:, 8] - marks[:, 0]
    span = marks[:, 8].max() - marks[:, 0].min()
    print(f'round {r}: {len(t)} waves, launch span {span} cycles, wave life median {np.median(life):.0f} '
          f'mean {life.mean():.0f}')
    for c in np.unique(code):
        sel = code == c
        bits = [nm for b, nm in ((1, 'noise'), (2, 'rank1'), (4, 'fullfactor'), (8, 'reuse'), (16, 'solve'),
                                 (32, 'lz-ok'), (64, 'lz-back'), (128, 'lean'), (256, 'noise-lean')) if c & b]
        ph = PHASES_LEAN if c & 128 else phases
        row = ' '.join(f'{nm} {np.mean(dt[sel, i]):7.0f}' for i, nm in enumerate(ph))
        print(f'code {c:3d} ({"+".join(bits) or "-"}): {sel.sum():6d} waves, life {np.mean(life[sel]):7.0f}: {row}')
    # concurrency: waves alive over the launch
    print('mean phase share of wave life:',
          ' '.join(f'{nm} {np.sum(dt[:, i]) / np.sum(life):.3f}' for i, nm in enumerate(phases)))


if __name__ == '__main__':
    main()
