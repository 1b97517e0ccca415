"""Build libgfd.so (the HIP/gfx950 C-ABI library) in-tree with hipcc.

    python -m gfd.build            # from gnn-fraud-detection_amd/

Each ``csrc/*.hip`` is compiled to an object in parallel, then linked into
``gfd/libgfd.so`` next to this file (git-ignored, shipped to the GPU box by the
gpurun snapshot).  ``--all`` (the driver's ``build()``) also builds the shipped
variants: ``libgfd_checked.so``, the bounds-checked diagnostic build.  No torch
involvement: the library is plain HIP + rocPRIM headers.

Provenance: every library carries ``gfd_build_id()`` = the SHA-256 of its
sources and headers (contents, not mtimes) with the compiler flags and target.
A library is rebuilt -- every object, from scratch -- unless the id it carries
equals the id of the sources next to it, so a shipped prebuilt library is
either provably built from this tree or replaced (``source_id`` /
``library_id``).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
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
# Per-source flags: {"file.hip": [flags]}
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


def _object_id(src: str, flags) -> str:
    """Content hash of what one object is compiled from: the source, every
    header, the flags and the target."""
    h = hashlib.sha256()
    for p in [src] + sorted(_deps()):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(list(flags) + SOURCE_FLAGS.get(os.path.basename(src), [])).encode())
    h.update(ARCH.encode())
    return h.hexdigest()


def _compile(src: str, objdir: str, flags) -> str:
    obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
    oid = _object_id(src, flags)
    stamp = obj + ".sha256"
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read().strip() == oid:
        return obj   # built from exactly these bytes
    cmd = [HIPCC, *flags, *SOURCE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    with open(stamp, "w") as f:
        f.write(oid + "\n")
    return obj


ID_TAG = "gfd-src-sha256:"


def source_id(flags=None) -> str:
    """SHA-256 over the library's sources and headers (relative path + bytes,
    sorted), the compile flags and the target: what gfd_build_id() returns."""
    h = hashlib.sha256()
    for p in sorted(sources() + _deps()):
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags if flags is not None else FLAGS).encode())
    h.update(ARCH.encode())
    return h.hexdigest()


def library_id(lib: str = None):
    """The source id a built library carries (read from the file; no dlopen)."""
    lib = lib or LIB
    try:
        data = open(lib, "rb").read()
    except OSError:
        return None
    i = data.find(ID_TAG.encode())
    return data[i + len(ID_TAG):i + len(ID_TAG) + 64].decode() if i >= 0 else None


def needs_build(lib: str = None, flags=None) -> bool:
    lib = lib or LIB
    return library_id(lib) != source_id(flags)


def _id_object(objdir: str, flags) -> str:
    """A one-function object carrying the source id (gfd_build_id)."""
    sid = source_id(flags)
    src = os.path.join(objdir, "gfd_build_id.hip")
    with open(src, "w") as f:
        f.write(f'extern "C" const char* gfd_build_id(void) {{ return "{ID_TAG}{sid} {ARCH}"; }}\n')
    obj = src[:-4] + ".o"
    r = subprocess.run([HIPCC, *flags, "-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for the build id:\n{r.stderr[-3000:]}")
    return obj


def _build_one(lib: str, objdir: str, flags, force: bool, verbose: bool) -> str:
    stale = needs_build(lib, flags)
    if not force and not stale:
        return lib
    os.makedirs(objdir, exist_ok=True)
    srcs = sources()   # (each object rebuilt unless its content stamp matches)
    workers = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir, flags), srcs))
    objs.append(_id_object(objdir, flags))
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
