"""Build liborbx.so (HIP, gfx950) in-tree with hipcc.

    python -m orbslam2commentedbyxcm_amd.build        # incremental
    python -m orbslam2commentedbyxcm_amd.build --clean

The shared library lands next to this file so that it travels with the repository
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).  Every translation
unit is compiled with -ffp-contract=off, and fuses exactly where the reference's g++
-O3 -march=native build fuses, with explicit fma (g++ contracts C++ even under
-std=c++11; measured on the reference's own BowVector.cpp): the descriptor / fastAtan2 /
projection float expressions must round identically (hazard H4).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "_obj"
LIB = PKG / "liborbx.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ORBX_ARCH", "gfx950")

SOURCES = ["orbx_geometry.cpp", "orbx_extract.hip", "orbx_match.hip", "orbx_api.cpp", "orbx_matcher.cpp", "orbx_vocab.hip", "orbx_bow.hip", "orbx_frame.hip", "orbx_fuse.hip", "orbx_runtime.cpp"]
HEADERS = ["orbx_sincos.h", "orbx_block_sort.h", "orbx_geometry.h", "orbx_kernels.h", "orbx_match_types.h", "orbx_error.h", "orb_pattern.inc", "orbx_gmem.h"]
FLAGS = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         f"-I{ROOT / 'include'}", f"-I{CSRC}"]


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _compile(src: str) -> Path:
    out = OBJ / (src + ".o")
    deps = [CSRC / src, ROOT / "include" / "orbx.h"] + [CSRC / h for h in HEADERS]
    if _newer(out, deps):
        cmd = [HIPCC, *FLAGS, "-c", str(CSRC / src), "-o", str(out)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
    return out


def build(verbose: bool = False) -> Path:
    OBJ.mkdir(exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(4, len(SOURCES))) as pool:
        objs = list(pool.map(_compile, SOURCES))
    if _newer(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(LIB), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


def build_variant(tag: str, defines: list[str]) -> Path:
    """A/B build: the same sources with extra -D defines into _ab/liborbx_<tag>.so (load
    it with ORBX_LIB=...; tools/ab.sh, tools/ab_args.sh)."""
    out_dir = CSRC.parent / "_ab"
    obj = out_dir / f"obj_{tag}"
    obj.mkdir(parents=True, exist_ok=True)
    flags = FLAGS + [f"-D{d}" for d in defines]

    def comp(src):
        out = obj / (src + ".o")
        r = subprocess.run([HIPCC, *flags, "-c", str(CSRC / src), "-o", str(out)], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
        return out

    with cf.ThreadPoolExecutor(max_workers=4) as pool:
        objs = list(pool.map(comp, SOURCES))
    lib = out_dir / f"liborbx_{tag}.so"
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(lib), *map(str, objs)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return lib


def clean() -> None:
    shutil.rmtree(OBJ, ignore_errors=True)
    LIB.unlink(missing_ok=True)


if __name__ == "__main__":
    if "--variant" in sys.argv:  # python -m orbslam2commentedbyxcm_amd.build --variant TAG -DNAME=V ...
        i = sys.argv.index("--variant")
        print(build_variant(sys.argv[i + 1], [a[2:] for a in sys.argv[i + 2:] if a.startswith("-D")]))
        sys.exit(0)
    if "--clean" in sys.argv:
        clean()
    build(verbose=True)
