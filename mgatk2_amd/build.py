"""Build the native libraries in-tree.

* ``mgatk2_amd/_lib/libmgpileup.so`` — HIP engine + C-ABI, gfx950 only
  (``hipcc --offload-arch=gfx950``), linked against RCCL.
* ``mgatk2_amd/_lib/libmgphost.so`` — host-side BAM ingest (g++, zlib).
* ``oracle/_build/liboracle.so`` — the CPU restatement (test infrastructure).
* ``oracle/_ref/`` is not built: the reference is pure Python (no native path
  to compile); its outputs are pinned through tests/golden/ instead.
"""

from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "mgatk2_amd"
CSRC = PKG / "csrc"
LIB_DIR = PKG / "_lib"
ENGINE_SO = LIB_DIR / "libmgpileup.so"
HOST_SO = LIB_DIR / "libmgphost.so"
ORACLE_DIR = ROOT / "oracle"
ORACLE_SO = ORACLE_DIR / "_build" / "liboracle.so"

HIP_SOURCES = ["mgp_engine.hip", "mgp_synth.hip", "mgp_txtgz.hip"]
HIP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-function"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (need ROCm for gfx950)")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_engine(force: bool = False, verbose: bool = False, out: Path | None = None,
                 defines: tuple[str, ...] = ()) -> Path:
    target = Path(out) if out else ENGINE_SO
    deps = [CSRC / s for s in HIP_SOURCES] + [CSRC / "mgp_kernels.h", CSRC / "mgp_txtgz.h", ROOT / "include" / "mgpileup.h"]
    if force or _stale(target, deps):
        LIB_DIR.mkdir(parents=True, exist_ok=True)
        tmp = target.with_suffix(".so.tmp")
        cmd = [_hipcc(), *HIP_FLAGS, *[f"-D{d}" for d in defines], *[str(CSRC / s) for s in HIP_SOURCES],
               "-o", str(tmp), "-lrccl"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True, cwd=str(CSRC))
        os.replace(tmp, target)
    return target


def build_host(force: bool = False, verbose: bool = False) -> Path:
    """libmgphost.so: native BAM ingest (include/mgpileup_host.h), plain C++ + zlib."""
    srcs = [CSRC / "host" / "mgp_bam.cpp", CSRC / "host" / "mgp_txt.cpp", CSRC / "host" / "mgp_tiles.cpp",
            CSRC / "host" / "mgp_bamw.cpp", CSRC / "host" / "mgp_shard.cpp", CSRC / "host" / "mgp_place.cpp",
            CSRC / "host" / "mgp_repack.cpp", CSRC / "host" / "mgp_route.cpp"]
    deps = srcs + [ROOT / "include" / "mgpileup_host.h", ROOT / "include" / "mgpileup.h",
                   CSRC / "host" / "mgp_pack32_host.h", CSRC / "host" / "mgp_place.h",
                   CSRC / "host" / "mgp_zcodec.h", CSRC / "host" / "mgp_pool.h"]
    if force or _stale(HOST_SO, deps):
        LIB_DIR.mkdir(parents=True, exist_ok=True)
        tmp = HOST_SO.with_suffix(".so.tmp")
        cxx = shutil.which("g++") or "c++"
        cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-pthread", f"-I{ROOT / 'include'}",
               *[str(s) for s in srcs], "-o", str(tmp), "-lz", "-ldl"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(tmp, HOST_SO)
    return HOST_SO


def build_oracle(force: bool = False, verbose: bool = False) -> Path:
    deps = [ORACLE_DIR / "mgp_oracle.c", ROOT / "include" / "mgpileup.h"]
    if force or _stale(ORACLE_SO, deps):
        ORACLE_SO.parent.mkdir(parents=True, exist_ok=True)
        tmp = ORACLE_SO.with_suffix(".so.tmp")
        cc = shutil.which("gcc") or "cc"
        cmd = [cc, "-O2", "-std=c11", "-fPIC", "-shared", "-Wall", str(ORACLE_DIR / "mgp_oracle.c"), "-o", str(tmp)]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(tmp, ORACLE_SO)
    return ORACLE_SO


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_engine(force, verbose)
    build_host(force, verbose)
    build_oracle(force, verbose)


if __name__ == "__main__":
    import sys

    build_all(force="--force" in sys.argv, verbose=True)
