"""In-tree build of libsurprise_amd.so for gfx950 (MI355X).

``hipcc`` cross-compiles without a GPU, so this runs in the CPU container too.
The output lives next to this file so it travels with the repo snapshot to the
GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(_HERE, "csrc", "mf_kernels.hip")
HDR = os.path.join(os.path.dirname(_HERE), "include", "surprise_amd.h")
OUT = os.path.join(_HERE, "libsurprise_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SURPRISE_AMD_ARCH", "gfx950")


def build(force: bool = False, verbose: bool = False) -> str:
    newest = max(os.path.getmtime(SRC), os.path.getmtime(HDR))
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= newest:
        return OUT
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
