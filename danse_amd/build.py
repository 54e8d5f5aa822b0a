"""In-tree build of the HIP extension (gfx950): ``libdanse_mi355x.so``.

``hipcc -c -fPIC`` of ``csrc/danse_engine.hip`` (online engine, C-ABI, bcast /
operator kernels), ``csrc/batch.hip`` (batch-mode engine), ``csrc/dxcp.hip`` (DXCP-PhaT SRO
estimator), ``csrc/tz.hip`` (T(z) few-samples compression), ``csrc/metrics.hip``
(SNR / fwSNRseg), ``csrc/stoi.hip`` ((e)STOI) and of
``csrc/update_class.hip`` once per filter-size class
(``-DDANSE_DMAX=N``, N = 1..12, 16, 20 and 24..64 in steps of 8, see
``csrc/classes.hpp``), in parallel, then one
``hipcc -shared`` link.  Objects go to ``danse_amd/_obj/``; the library sits
next to this file so that it travels with the repository snapshot to the GPU
box.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / 'csrc'
OBJ = HERE / '_obj'
OUT = HERE / 'libdanse_mi355x.so'
INC = HERE.parent / 'include'
CLASSES = list(range(1, 13)) + [16, 20, 24, 32, 40, 48, 56, 64]
LANE_MAX_D = 12   # csrc/classes.hpp kLaneMaxD
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC']


def _units():
    """(object name, source, extra flags) of every translation unit."""
    u = [('danse_engine.o', CSRC / 'danse_engine.hip', []), ('batch.o', CSRC / 'batch.hip', []),
         ('dxcp.o', CSRC / 'dxcp.hip', []), ('tz.o', CSRC / 'tz.hip', []),
         ('metrics.o', CSRC / 'metrics.hip', []), ('stoi.o', CSRC / 'stoi.hip', []),
         ('scene.o', CSRC / 'scene.hip', []), ('resident.o', CSRC / 'resident.hip', []),
         ('wide.o', CSRC / 'wide.hip', [])]
    for n in CLASSES:
        # lane-per-bin classes: no SLP packing of the float32 complex math
        # (the packed pairs need swapped operand copies; with them the eigen
        # kernel spills to scratch, without them it fits the register file)
        extra = ['-fno-slp-vectorize'] if n <= LANE_MAX_D else []
        u.append((f'update_d{n}.o', CSRC / 'update_class.hip', [f'-DDANSE_DMAX={n}', *extra]))
    return u


def _deps(src: Path, seen=None) -> set:
    """The quoted #includes of a source, recursively (per-unit staleness, so a
    broadcast-kernel edit does not recompile every solver class)."""
    seen = set() if seen is None else seen
    for line in src.read_text().splitlines():
        line = line.strip()
        if line.startswith('#include "'):
            dep = (src.parent / line.split('"')[1]).resolve()
            if dep.exists() and dep not in seen:
                seen.add(dep)
                _deps(dep, seen)
    return seen


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *_deps(src)])


# A/B variants of the same library (compile-time switches; loaded with
# DANSE_LIB=danse_amd/libdanse_<name>.so): objects in _obj/<name>/
VARIANTS = {
    'stamp': ['-DDANSE_STAMP=1'],   # per-wave phase clocks in update_kernel_2d (DANSE_UPDATE_TRACE)
    'nodma': ['-DDANSE_LEAN_DMA=0'],   # update_kernel_2dc's factor record through VGPRs
    'lz6': ['-DDANSE_LEAN_LZ_VAD_DELTA=-2'],   # update_kernel_2dc: six Lanczos steps on VAD frames
    'lzlocal': ['-DDANSE_LZ_FULL_REORTH=0'],   # Lanczos reorthogonalised against the last two vectors only
}


MARK = b'DANSE_SRC_HASH:'


def source_hash(variant: str | None = None) -> str:
    """sha256 over every HIP / C++ source and header of the library, the
    compile flags and the size classes.  build() embeds it in the library
    (``danse_mi355x_build_id``); ``_lib.load_library`` refuses a library whose
    id differs from the sources next to it, so a shipped ``.so`` is provably
    the build of the shipped sources."""
    h = hashlib.sha256()
    files = sorted([*CSRC.glob('*.hip'), *CSRC.glob('*.hpp'), *INC.glob('*.h')])
    for f in files:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    h.update(repr((FLAGS, CLASSES, VARIANTS.get(variant) if variant else None)).encode())
    return h.hexdigest()


def embedded_hash(lib: Path) -> str | None:
    """The source hash a built library carries (None: none)."""
    try:
        b = lib.read_bytes()
    except OSError:
        return None
    i = b.find(MARK)
    return b[i + len(MARK):i + len(MARK) + 64].decode() if i >= 0 else None


def _paths(variant):
    if variant is None:
        return OBJ, OUT
    return OBJ / variant, HERE / f'libdanse_{variant}.so'


def up_to_date(variant: str | None = None) -> bool:
    obj, out = _paths(variant)
    if not out.exists():
        return False
    return embedded_hash(out) == source_hash(variant)


def build(force: bool = False, verbose: bool = True, jobs: int | None = None, variant: str | None = None) -> Path:
    obj, out = _paths(variant)
    if not force and up_to_date(variant):
        return out
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    obj.mkdir(parents=True, exist_ok=True)
    vflags = VARIANTS[variant] if variant else []
    todo = [(o, s, x) for o, s, x in _units() if force or _stale(obj / o, s)]

    def compile_one(item):
        o, s, x = item
        cmd = [hipcc, *FLAGS, f'-I{INC}', *vflags, *x, '-c', str(s), '-o', str(obj / o) + '.tmp']
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed for {o}:\n{r.stderr}')
        os.replace(str(obj / o) + '.tmp', obj / o)

    n = jobs or min(16, os.cpu_count() or 4, max(1, len(todo)))
    # heaviest classes first so the pool drains evenly
    todo.sort(key=lambda it: -int(it[0][8:-2]) if it[0].startswith('update_d') else 0)
    with ThreadPoolExecutor(max_workers=n) as ex:
        list(ex.map(compile_one, todo))
    # the build id: the source hash as a string and an exported C function
    sh = source_hash(variant)
    bid = obj / 'build_id.cpp'
    bid.write_text('// generated by danse_amd/build.py\n'
                   f'static const char kId[] = "{MARK.decode()}{sh}";\n'
                   'extern "C" __attribute__((visibility("default"))) const char* danse_mi355x_build_id() '
                   '{ return kId + ' + str(len(MARK)) + '; }\n')
    subprocess.run(['g++', '-O2', '-fPIC', '-c', str(bid), '-o', str(obj / 'build_id.o')], check=True)
    cmd = [hipcc, '--offload-arch=gfx950', '-fPIC', '-shared', *[str(obj / o) for o, _, _ in _units()],
           str(obj / 'build_id.o'), '-o', str(out) + '.tmp']
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(str(out) + '.tmp', out)
    return out


if __name__ == '__main__':
    _v = [a.split('=', 1)[1] for a in sys.argv[1:] if a.startswith('--variant=')]
    build(force='--force' in sys.argv, variant=_v[0] if _v else None)
