"""In-tree build of the HIP extension (gfx950): ``libdanse_mi355x.so``.

Plain ``hipcc -shared -fPIC`` of ``csrc/danse_engine.hip`` (kernels in
``csrc/*.hpp``); the output sits next to this file so that it travels with the
repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / 'csrc' / 'danse_engine.hip'
OUT = HERE / 'libdanse_mi355x.so'
INC = HERE.parent / 'include'


def _sources():
    return [SRC] + sorted((HERE / 'csrc').glob('*.hpp')) + [INC / 'danse_mi355x.h']


def up_to_date() -> bool:
    if not OUT.exists():
        return False
    t = OUT.stat().st_mtime
    return all(s.stat().st_mtime <= t for s in _sources())


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and up_to_date():
        return OUT
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    cmd = [hipcc, '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-shared',
           f'-I{INC}', str(SRC), '-o', str(OUT) + '.tmp']
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(str(OUT) + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
