"""Build librpt.so (HIP kernels for gfx950 + host runtime) in-tree with hipcc.

No CMake, no torch extension machinery: every ``csrc/*.hip`` / ``csrc/*.cpp`` is compiled to an
object with ``hipcc --offload-arch=gfx950`` and linked into ``rpt/librpt.so``.  Objects are
rebuilt only when a source or header is newer, and all of them when the build stamp (hipcc
version, flags, offload arch) differs from the one recorded in ``build/STAMP``.
``-ffp-contract=off`` is global: the parity
contract (bit-identical labels and centroids) forbids FMA contraction of the reference's
separately rounded float operations.

``build(ab=True)`` (``python -m rpt._build --ab``) compiles the same sources with ``-DRPT_AB``
into ``rpt/librpt_ab.so`` (objects under ``build_ab/``): the only build whose kernels read the
``RPT_*`` A/B switches from the environment (csrc/common.h ``ab_env``).  ``tools/ab_*.sh`` load it
through ``RPT_LIB``; the shipped ``librpt.so`` ignores the environment.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR.parent / "csrc"
INCLUDE = PKG_DIR.parent.parent / "include"
BUILD = PKG_DIR.parent / "build"
LIB = PKG_DIR / "librpt.so"
BUILD_AB = PKG_DIR.parent / "build_ab"
LIB_AB = PKG_DIR / "librpt_ab.so"

ARCH = os.environ.get("RPT_OFFLOAD_ARCH", "gfx950")
COMMON_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=off",
    "-fno-math-errno",
    f"--offload-arch={ARCH}",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-result",
    f"-I{INCLUDE}",
    f"-I{CSRC}",
]


def _hipcc() -> str:
    exe = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(exe).exists():
        raise RuntimeError("hipcc not found: the ROCm toolchain is required to build librpt")
    return exe


def _sources() -> list[Path]:
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _headers_mtime() -> float:
    # (*.inc: kernel sources included by one .hip, e.g. the A/B-only stdbscan_ab.inc)
    hs = list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, obj: Path, extra=()) -> str:
    cmd = [_hipcc(), *COMMON_FLAGS, *extra, "-c", str(src), "-o", str(obj)]
    if src.suffix == ".cpp":
        cmd.insert(1, "-x")
        cmd.insert(2, "hip")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return r.stderr


def _stamp(extra=()) -> str:
    r = subprocess.run([_hipcc(), "--version"], capture_output=True, text=True)
    return "\n".join([r.stdout.strip(), " ".join([*COMMON_FLAGS, *extra]), ARCH]) + "\n"


def build(verbose: bool = False, force: bool = False, jobs: int | None = None,
          ab: bool = False) -> Path:
    extra = ("-DRPT_AB",) if ab else ()
    build_dir, lib = (BUILD_AB, LIB_AB) if ab else (BUILD, LIB)
    build_dir.mkdir(parents=True, exist_ok=True)
    stamp_file = build_dir / "STAMP"
    stamp = _stamp(extra)
    if not stamp_file.exists() or stamp_file.read_text() != stamp:
        force = True  # other flags, arch or compiler: objects built before are stale
    hdr_t = _headers_mtime()
    todo = []
    objs = []
    for src in _sources():
        obj = build_dir / (src.name + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_t):
            todo.append((src, obj))
    jobs = jobs or min(8, max(1, os.cpu_count() or 1))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for (src, _), warn in zip(todo, ex.map(lambda a: _compile(*a, extra), todo)):
            if verbose and warn.strip():
                print(f"[rpt build] {src.name}:\n{warn}")
    if todo or not lib.exists():
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib),
               *[str(o) for o in objs]]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link of {lib.name} failed:\n{r.stderr}")
    stamp_file.write_text(stamp)
    if verbose:
        print(f"[rpt build] {lib} ({len(todo)} objects rebuilt)")
    return lib


if __name__ == "__main__":
    import sys

    build(verbose=True, ab="--ab" in sys.argv[1:])
