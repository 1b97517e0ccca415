"""Build libgfd.so (the HIP/gfx950 C-ABI library) in-tree with hipcc.

    python -m gfd.build            # from gnn-fraud-detection_amd/

Each ``csrc/*.hip`` is compiled to an object in parallel, then linked into
``gfd/libgfd.so`` next to this file (git-ignored, shipped to the GPU box by the
gpurun snapshot).  ``--all`` (the driver's ``build()``) also builds the shipped
variants: ``libgfd_checked.so``, the bounds-checked diagnostic build.  Rebuilds
only when a source or header is newer than the library.  No torch involvement: the library is plain HIP + rocPRIM headers.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                       # gnn-fraud-detection_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
# GFD_BUILD_VARIANT=<name>: a diagnostic / A-B build (with GFD_EXTRA_FLAGS) into
# libgfd_<name>.so / build/obj_<name>; the product library is untouched.
VARIANT = os.environ.get("GFD_BUILD_VARIANT", "")
if os.environ.get("GFD_EXTRA_FLAGS") and not VARIANT:
    raise RuntimeError("GFD_EXTRA_FLAGS needs GFD_BUILD_VARIANT (never rebuild libgfd.so with A/B flags)")
ARCH = os.environ.get("GFD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
# -fno-honor-nans: fmaxf without operand canonicalisation, so the DPP row
# rotations fold into v_max_f32_dpp (no kernel relies on NaN semantics)
BASE_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              "-fno-honor-nans",
              f"-I{INCLUDE}", f"-I{CSRC}", "-Wall", "-Wno-unused-function"]
# the variants build() always produces next to the product library:
#   checked -- the bounds-checked diagnostic build (gfd_check.h)
SHIPPED_VARIANTS = {"checked": ["-DGFD_CHECKED"]}
# Per-source flags (none at present): {"file.hip": [flags]}
SOURCE_FLAGS = {}


def lib_path(variant: str = "") -> str:
    return os.path.join(PKG, f"libgfd_{variant}.so" if variant else "libgfd.so")


def obj_dir(variant: str = "") -> str:
    return os.path.join(ROOT, "build", f"obj_{variant}" if variant else "obj")


# the library this process builds by default (env-selected A/B variant or the product)
LIB = lib_path(VARIANT)
OBJDIR = obj_dir(VARIANT)
FLAGS = BASE_FLAGS + os.environ.get("GFD_EXTRA_FLAGS", "").split()


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return hdrs


def _compile(src: str, objdir: str, flags) -> str:
    obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
    newest = max(os.path.getmtime(p) for p in [src] + _deps())
    if os.path.exists(obj) and os.path.getmtime(obj) >= newest:
        return obj
    cmd = [HIPCC, *flags, *SOURCE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj


def needs_build(lib: str = None) -> bool:
    lib = lib or LIB
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in sources() + _deps())


def _build_one(lib: str, objdir: str, flags, force: bool, verbose: bool) -> str:
    if not force and not needs_build(lib):
        return lib
    os.makedirs(objdir, exist_ok=True)
    srcs = sources()
    workers = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir, flags), srcs))
    tmp = lib + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, lib)
    if verbose:
        print(f"[gfd.build] built {lib} from {len(srcs)} sources for {ARCH}", file=sys.stderr)
    return lib


def build(force: bool = False, verbose: bool = True) -> str:
    """The library this process selects (the product, or GFD_BUILD_VARIANT)."""
    return _build_one(LIB, OBJDIR, FLAGS, force, verbose)


def build_all(force: bool = False, verbose: bool = True) -> list:
    """The product library and every shipped variant (the driver's build())."""
    out = [_build_one(lib_path(), obj_dir(), BASE_FLAGS, force, verbose)]
    for name, extra in SHIPPED_VARIANTS.items():
        out.append(_build_one(lib_path(name), obj_dir(name), BASE_FLAGS + extra, force, verbose))
    return out


if __name__ == "__main__":
    if "--all" in sys.argv:
        build_all(force="--force" in sys.argv)
    else:
        build(force="--force" in sys.argv)
