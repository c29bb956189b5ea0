"""In-tree build of librs_hip.so (hipcc, gfx950 only).

Every ``csrc/*.hip`` / ``csrc/*.cpp`` is compiled to an object with
``hipcc --offload-arch=gfx950`` (in parallel) and linked into
``recommender_system_amd/librs_hip.so``.  The library is rebuilt only when a
source, header or this file is newer than it.  The .so is git-ignored but
travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
LIB = PKG / "librs_hip.so"
OBJDIR = PKG / "build"
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build librs_hip.so)")


def sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _deps_mtime() -> float:
    files = sources() + list(CSRC.glob("*.hpp")) + list(INCLUDE.glob("*.h")) + [Path(__file__)]
    return max(f.stat().st_mtime for f in files)


def up_to_date() -> bool:
    return LIB.exists() and LIB.stat().st_mtime >= _deps_mtime()


def _compile(src: Path, hipcc: str, extra) -> Path:
    obj = OBJDIR / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _headers_mtime()):
        return obj
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
           "-Wno-unused-function", "-I", str(INCLUDE), "-I", str(CSRC), "-c", str(src),
           "-o", str(obj)] + list(extra)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def _headers_mtime() -> float:
    files = list(CSRC.glob("*.hpp")) + list(INCLUDE.glob("*.h")) + [Path(__file__)]
    return max(f.stat().st_mtime for f in files)


def build(force: bool = False, verbose: bool = True, extra_flags=()) -> Path:
    if not force and up_to_date():
        return LIB
    hipcc = _hipcc()
    OBJDIR.mkdir(exist_ok=True)
    if force:
        for o in OBJDIR.glob("*.o"):
            o.unlink()
    srcs = sources()
    jobs = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hipcc, extra_flags), srcs))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"[recommender_system_amd] built {LIB} from {len(srcs)} sources", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
