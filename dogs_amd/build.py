"""Builds libdogs_hip.so in-tree (dogs_amd/_lib/) for gfx950 with hipcc.  No torch extension machinery:
the library is a plain C-ABI shared object (include/dogs_hip.h) loaded with ctypes."""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(OUT_DIR, "libdogs_hip.so")
SOURCES = ["sortscan.hip", "raster_fwd.hip", "raster_bwd.hip", "aux_kernels.hip", "optim.hip", "export.hip", "loader.hip", "blocksplit.hip",
           "colmap.hip", "mask_conv.hip", "mask_head.hip", "capi.hip"]
ARCH = os.environ.get("DOGS_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off + explicit fmaf and correctly rounded div/sqrt: the bit-exact key contract with the
# CPU oracle (DESIGN.md "Bit-exact keys").
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wno-unused-result", "-munsafe-fp-atomics"]


def _hipcc() -> str:
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found: the gfx950 library cannot be built")
    return h


def _stale(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(HERE, "..", "include", "dogs_hip.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    hipcc = _hipcc()
    jobs = []
    objs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OUT_DIR, s.replace(".hip", ".o"))
        objs.append(obj)
        if force or _stale(obj, src):
            jobs.append([hipcc, *FLAGS, "-c", src, "-o", obj])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr, file=sys.stderr)

    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if jobs or not os.path.exists(LIB):
        run([hipcc, *FLAGS, "-shared", "-o", LIB, *objs])
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
