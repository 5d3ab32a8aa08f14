"""Build libdivrec_hip.so (the C-ABI HIP library) in-tree for gfx950.

    python diversity-recommendations_amd/build_native.py [--jobs N] [--verbose]

Each csrc/*.hip file is compiled to an object with hipcc --offload-arch=gfx950
(cross-compiles without a GPU), then linked into divrec/_lib/libdivrec_hip.so.
Objects are rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent
if str(PKG_ROOT) not in sys.path:
    sys.path.insert(0, str(PKG_ROOT))
from divrec._buildid import source_hash  # noqa: E402  (no torch import)

CSRC = PKG_ROOT / "csrc"
INCLUDE = PKG_ROOT.parent / "include"
OBJ_DIR = PKG_ROOT / "build" / "obj"
LIB_DIR = PKG_ROOT / "divrec" / "_lib"
LIB_PATH = LIB_DIR / "libdivrec_hip.so"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-munsafe-fp-atomics",
    f"-I{INCLUDE}",
    f"-I{CSRC}",
]


# Per-source flags. ild.hip: MFMA results in VGPRs (the streamed ILD's
# epilogue reads every Gram element once with VALU; AGPR results each need a
# v_accvgpr_read first).
FILE_FLAGS = {"ild.hip": ("-mllvm", "-amdgpu-mfma-vgpr-form")}


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, verbose: bool, obj_dir: Path = OBJ_DIR, extra=(), build_id: str = "") -> Path:
    obj = obj_dir / (src.stem + ".o")
    stamp = obj_dir / "flags.txt"
    same_flags = stamp.exists() and stamp.read_text() == " ".join(extra)
    id_flags = ()
    if src.name == "capi.hip":  # the translation unit that carries the build id
        id_flags = (f'-DDR_BUILD_ID="{build_id}"',)
        id_stamp = obj_dir / "build_id.txt"
        same_flags = same_flags and id_stamp.exists() and id_stamp.read_text() == build_id
    if same_flags and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime,
                                                                  _headers_mtime()):
        return obj
    cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(src.name, ()), *extra, *id_flags, "-c", str(src), "-o",
           str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int = 4, verbose: bool = False, diag: bool = False, variant: str = "",
          defines=()) -> Path:
    """Build the product library; with diag=True the instrumented
    libdivrec_hip_diag.so (-DDR_TOPK_DIAG); with variant=NAME and defines
    (KEY=VAL strings) libdivrec_hip_NAME.so for tools/variant_bench.py. Diag
    and variant libraries are measurement tools: the product path loads them
    only when DIVREC_HIP_LIB points at one."""
    defines = tuple(defines)
    if diag:
        variant, defines = variant or "diag", ("DR_TOPK_DIAG",) + defines
    obj_dir = OBJ_DIR.parent / f"obj_{variant}" if variant else OBJ_DIR
    lib_path = LIB_DIR / f"libdivrec_hip_{variant}.so" if variant else LIB_PATH
    extra = tuple(f"-D{d}" for d in defines)
    obj_dir.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    build_id = source_hash()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose, obj_dir, extra, build_id), srcs))
    (obj_dir / "flags.txt").write_text(" ".join(extra))
    (obj_dir / "build_id.txt").write_text(build_id)
    newest = max(o.stat().st_mtime for o in objs)
    if lib_path.exists() and lib_path.stat().st_mtime >= newest:
        return lib_path
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, lib_path)
    return lib_path


PEAKS_SRC = PKG_ROOT.parent / "tools" / "peaks.hip"
PEAKS_LIB = PKG_ROOT.parent / "tools" / "_peaks" / "libdivrec_peaks.so"


def build_peaks(verbose: bool = False) -> Path:
    """tools/peaks.hip -> tools/_peaks/libdivrec_peaks.so: the achievable-peak
    probes bench.py reports beside the vendor peaks (measurement only, not
    part of the product library)."""
    PEAKS_LIB.parent.mkdir(parents=True, exist_ok=True)
    if PEAKS_LIB.exists() and PEAKS_LIB.stat().st_mtime >= PEAKS_SRC.stat().st_mtime:
        return PEAKS_LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-shared",
           str(PEAKS_SRC), "-o", str(PEAKS_LIB)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for peaks.hip:\n{r.stdout}\n{r.stderr}")
    return PEAKS_LIB


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--diag", action="store_true", help="build the instrumented diag library")
    ap.add_argument("--variant", default="", help="build libdivrec_hip_<NAME>.so")
    ap.add_argument("-D", dest="defines", action="append", default=[],
                    help="KEY=VAL preprocessor define for a variant build (repeatable)")
    args = ap.parse_args()
    path = build(args.jobs, args.verbose, args.diag, args.variant, args.defines)
    print(path)
    if not args.variant and not args.diag:
        print(build_peaks(args.verbose))
    return 0


if __name__ == "__main__":
    sys.exit(main())
