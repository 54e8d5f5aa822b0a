"""Code-generation guards (CPU, hipcc cross-compiles gfx950): regressions that
parity tests cannot see but that cost the GPU dearly.

* The resident kernel's LDS hand-offs must stay ``ds_`` instructions: a
  laundered LDS pointer once turned them into flat accesses (DESIGN.md §5.3;
  that build faulted with an aperture violation).
* The hot update kernels must not use scratch: a struct copy of a
  register-array element to global memory, or an over-full register budget,
  silently moves arrays to scratch.  (That check
  compiles two size classes, about 3.5 minutes: opt-in, DANSE_ISA_FULL=1.)
* The broadcast, fewSamples and DXCP kernels must not use scratch either:
  their loads are issued as held straight runs, and a run
  too long for the registers spills.
"""
import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / 'danse_amd' / 'csrc'
HIPCC = shutil.which('hipcc') or '/opt/rocm/bin/hipcc'

pytestmark = pytest.mark.skipif(not Path(HIPCC).exists(), reason='hipcc not available')


def _device_asm(src, *defines):
    cmd = [HIPCC, '--offload-arch=gfx950', '-O3', '-std=c++17', f'-I{ROOT / "include"}', *defines,
           '--cuda-device-only', '-S', str(src), '-o', '-']
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def _functions(asm, pattern):
    """{mangled name: body} of the kernels whose name matches pattern."""
    out = {}
    for m in re.finditer(r'^(_Z[^:\s]+):', asm, re.M):
        name = m.group(1)
        if not re.search(pattern, name):
            continue
        end = asm.find(f'.Lfunc_end', m.end())
        out[name] = asm[m.end():end]
    return out


def _scratch_sizes(asm, pattern):
    """{kernel name: private segment bytes} from the code-object metadata."""
    sizes = {}
    for blk in re.split(r'\n\s+- \.', asm):
        nm = re.search(r'\.name:\s+(\S+)', blk)
        ps = re.search(r'\.private_segment_fixed_size:\s+(\d+)', blk)
        if nm and ps and re.search(pattern, nm.group(1)):
            sizes[nm.group(1)] = int(ps.group(1))
    return sizes


def test_resident_kernel_has_no_flat_accesses():
    asm = _device_asm(CSRC / 'resident.hip')
    fns = _functions(asm, r'resident_kernel')
    assert fns, 'resident_kernel not found in the device assembly'
    for name, body in fns.items():
        flat = [ln.strip() for ln in body.splitlines() if re.match(r'\s+flat_(load|store|atomic)', ln)]
        assert not flat, (name, flat[:5])


@pytest.mark.skipif(not os.environ.get('DANSE_ISA_FULL'),
                    reason='3.5 minutes of compiles: DANSE_ISA_FULL=1 runs it (the default CPU suite stays short)')
def test_update_kernels_use_no_scratch():
    # the N2 class (DMAX 40: lane grid G = 8) and config B's lane class (D = 11)
    for dmax, extra in ((40, []), (11, ['-fno-slp-vectorize'])):
        asm = _device_asm(CSRC / 'update_class.hip', f'-DDANSE_DMAX={dmax}', *extra)
        # (the GEVD kernels of the online engine: update_kernel_2d, and
        # update_kernel_lane<D, R, GEVD = true, *>; the MWF lane kernel keeps
        # two float64 triangles and spills at D = 11 -- not a config's path)
        sizes = _scratch_sizes(asm, r'^_ZN5danse(16update_kernel_2d|18update_kernel_laneILi\d+ELi\d+ELb1E)')
        assert sizes, f'no update kernels found for DMAX {dmax}'
        bad = {k: v for k, v in sizes.items() if v != 0}
        assert not bad, (dmax, bad)


def test_broadcast_and_dxcp_kernels_use_no_scratch():
    # the broadcast kernels hold five 16-element preload runs next to the FFT
    # registers; DXCP's state preloads spill at 16 per chunk
    asm = _device_asm(CSRC / 'danse_engine.hip')
    # (and the start-gate kernels: the per-lane form holds a float64 triangle
    # of up to 78 entries, the register form up to 13 per lane)
    sizes = _scratch_sizes(asm, r'bcast_kernel|fs_chunk_kernel|fs_ir_kernel|gate_kernel_lane|gate_kernel_reg')
    assert len(sizes) >= 11, sizes
    assert not {k: v for k, v in sizes.items() if v != 0}, sizes
    asm = _device_asm(CSRC / 'dxcp.hip')
    sizes = _scratch_sizes(asm, r'dxcp_kernel')
    assert sizes and not {k: v for k, v in sizes.items() if v != 0}, sizes
