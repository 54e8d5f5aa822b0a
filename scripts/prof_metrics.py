"""fwSNRseg and eSTOI on 64 pairs of 10 s signals (the E battery's
per-scene metric batch) for a rocprofv3 kernel-statistics run."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from danse_amd import metrics as DM  # noqa: E402

rng = np.random.default_rng(1)
B, T = 64, 160000
c = torch.from_numpy(rng.standard_normal((B, T))).cuda()
e = c * 0.9 + 0.3 * torch.from_numpy(rng.standard_normal((B, T))).cuda()
for _ in range(3):
    per, mean = DM.fwsnrseg_batch(c, e, 16000.0)
torch.cuda.synchronize()
print('frames', per.shape, 'mean[0]', float(mean[0]))
for _ in range(3):
    st = DM.stoi_batch(c, e, 16000, extended=True)
torch.cuda.synchronize()
print('estoi[0]', float(np.asarray(st.cpu() if hasattr(st, 'cpu') else st).ravel()[0]))
