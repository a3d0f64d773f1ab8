"""Build libpinot_amd.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m pinot_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = [os.path.join(HERE, "csrc", "kernels.hip"), os.path.join(HERE, "csrc", "host.cpp")]
DEPS = SRC + [os.path.join(HERE, "csrc", "device_types.h"), os.path.join(HERE, "..", "include", "pinot_amd.h")]
OUT = os.path.join(HERE, "libpinot_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-munsafe-fp-atomics",
         "-Wall", "-Wno-unused-parameter"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in DEPS)


def build(force: bool = False) -> str:
    if force or needs_build():
        cmd = [HIPCC, *FLAGS, *SRC, "-o", OUT]
        print("+", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
