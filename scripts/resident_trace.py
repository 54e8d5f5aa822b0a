"""Per-round timing of the resident engine (DANSE_RESIDENT_TRACE wall-clock
marks, csrc/resident.hpp): config B at S = 1, where the round's critical
path goes (broadcast waves, the updating node's update waves, hand-offs)."""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ['DANSE_RESIDENT_TRACE'] = '1'


def main():
    import torch
    import bench
    from danse_amd.engine import DanseEngine
    from danse_amd.scene import make_scene
    wl = bench.WORKLOADS['B']
    dp, wp = bench._wl_params(wl)
    sc = make_scene(wl['M'], sigDur=wl['dur'], seed=1000)
    sc.get_vad_per_frame(dp.DFTsize, dp.Ns, wp.vadMinProportionActive)
    eng = DanseEngine([sc], dp, vadMinProp=wp.vadMinProportionActive, resident=True)
    for _ in range(3):
        eng.run()
    torch.cuda.synchronize()
    nb = ctypes.c_size_t(0)
    eng.lib.danse_engine_resident_trace(eng.eng, None, ctypes.byref(nb))
    tr = np.zeros(nb.value // 8, dtype=np.uint64)
    eng.lib.danse_engine_resident_trace(eng.eng, tr.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nb))
    K, R, F = eng.K, eng.R, eng.F
    FG = (F + 3) // 4
    grid = tr.size // (2 * R)
    tr = tr.reshape(R, grid, 2).astype(np.float64) * 10e-3   # us (100 MHz)
    nZ = K
    t0 = tr[0, nZ:, 0].min()
    tr = tr - t0
    zs, ze = tr[:, :nZ, 0], tr[:, :nZ, 1]
    us, ue = tr[:, nZ:, 0], tr[:, nZ:, 1]
    fl = eng.flags[:, 0, 0, :]
    solve = (fl & 0x10) != 0   # DANSE_FLAG_SOLVE
    print('round period (us): median %.2f' % np.median(np.diff(ue.max(axis=1))))
    rows = []
    for r in range(1, R - 1):
        upd = np.flatnonzero(solve[r])
        zlast = ze[r].max()
        ustart = us[r].min()
        uend_all = ue[r].max()
        uend_nonsolve = np.max([ue[r, k * FG:(k + 1) * FG].max() for k in range(K) if k not in upd]) if len(upd) < K else np.nan
        zwait_done = zs[r + 1].min() if r + 1 < R else np.nan
        rows.append((zlast - ze[r].min(), ustart - zlast, uend_all - ustart, uend_nonsolve - ustart, zwait_done - uend_all,
                     ze[r + 1].max() - zs[r + 1].min() if r + 1 < R else np.nan))
    a = np.array(rows)
    names = ['Z spread', 'Z publish -> U start', 'U round (all)', 'U round (non-solving nodes)', 'U end -> Z start',
             'Z work (next)']
    for i, n in enumerate(names):
        print(f'{n:32s} median {np.nanmedian(a[:, i]):8.2f} us  p90 {np.nanpercentile(a[:, i], 90):8.2f}')
    eng.close()


if __name__ == '__main__':
    main()
