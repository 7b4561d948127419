"""In-tree builder for the gfx950 HIP kernel library (``libdrn_kernels.so``).

Every ``csrc/kernels/*.hip`` translation unit is compiled by ``hipcc --offload-arch=gfx950``
into an object (in parallel, incrementally) and linked into one shared library next to this
file. The library exposes a plain C ABI (``DRN_API`` functions in csrc/) that the runtime
calls through ctypes with raw device pointers and the current HIP stream, so it does not link
against libtorch and compiles in seconds. At load time the HIP runtime symbol
``libamdhip64.so.7`` resolves to the copy PyTorch already loaded (same SONAME), so kernels and
torch share one runtime, one device context and one set of streams.

The reference has no native code at all; this replaces the cuDNN / MKL-DNN
kernels its TF1 graph dispatched to.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path
from typing import Optional

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "csrc"
KERNELS = CSRC / "kernels"
INCLUDE = CSRC / "include"
LIB_DIR = Path(__file__).resolve().parent
LIB_PATH = LIB_DIR / "libdrn_kernels.so"
HOST_LIB_PATH = LIB_DIR / "libdrn_host.so"
HOST_SRC = CSRC / "host"
OBJ_DIR = REPO / "build" / "obj"
ARCH = os.environ.get("DRN_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the gfx950 kernel library cannot be built")


def sources() -> list[Path]:
    return sorted(KERNELS.glob("*.hip"))


def source_hash(kernels: Path = KERNELS, include: Path = INCLUDE) -> str:
    """sha256 over every kernel source and shared header (relative name + bytes). Compiled into
    the library (drn_src_hash) and checked by ops._lib.lib(), so a library built from other
    sources is refused whatever the file times say."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(kernels.glob("*.hip")) + sorted(include.glob("*.h")):
        h.update(f.parent.name.encode() + b"/" + f.name.encode() + b"\0")
        h.update(f.read_bytes())
    return h.hexdigest()


# kernels whose code the tuner's choices depend on (the conv / weight-gradient / stem tiles and
# their fused prologues / epilogues, all through the shared headers)
TUNE_SOURCES = ("conv_fwd.hip", "conv_wgrad.hip", "stem.hip")


def tune_hash(kernels: Path = KERNELS, include: Path = INCLUDE) -> str:
    """sha256 over the sources the kernel-selection database depends on (TUNE_SOURCES + shared
    headers): the database section key (ops/tunedb.py), so an edit of a pooling / optimizer /
    BatchNorm-apply kernel does not throw away the shipped conv choices."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(kernels / n for n in TUNE_SOURCES) + sorted(include.glob("*.h")):
        h.update(f.parent.name.encode() + b"/" + f.name.encode() + b"\0")
        h.update(f.read_bytes())
    return h.hexdigest()


def _stamp_object() -> Path:
    """A translation unit returning source_hash() and tune_hash(), rebuilt when they change."""
    gen = OBJ_DIR / "drn_src_stamp.cc"
    text = ('extern "C" __attribute__((visibility("default"))) const char* drn_src_hash() '
            f'{{ return "{source_hash()}"; }}\n'
            'extern "C" __attribute__((visibility("default"))) const char* drn_tune_hash() '
            f'{{ return "{tune_hash()}"; }}\n')
    if not gen.exists() or gen.read_text() != text:
        gen.write_text(text)
    obj = gen.with_suffix(".o")
    if not obj.exists() or obj.stat().st_mtime < gen.stat().st_mtime:
        cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
        res = subprocess.run([cxx, "-O2", "-fPIC", "-c", str(gen), "-o", str(obj)], capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"source stamp build failed:\n{res.stderr[-2000:]}")
    return obj


def _compile(src: Path, extra: list[str], obj_dir: Optional[Path] = None, include: Path = INCLUDE) -> Path:
    obj = (obj_dir or OBJ_DIR) / (src.stem + ".o")
    hdr = max((h.stat().st_mtime for h in include.glob("*.h")), default=0.0)
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr):
        return obj
    # DRN_CONV_TRACE=1: diagnostics build with the per-workgroup conv timeline
    # (scripts/trace_conv.py); never the default -- the instrumentation costs ~2.5 % of a step
    trace = ["-DDRN_CONV_TRACE"] if os.environ.get("DRN_CONV_TRACE") == "1" else []
    trace += os.environ.get("DRN_HIPCC_EXTRA", "").split()  # A/B builds (e.g. -DDRN_KORDER_TAP_OUTER)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-I", str(include),
           "-Wno-unused-result", "-c", str(src), "-o", str(obj)] + trace + extra
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{res.stderr[-6000:]}")
    return obj


def build_host_sanitizer_driver(kind: str = "address", out_dir: Optional[str] = None) -> Path:
    """Build csrc/host/tests/host_sanitize_main.cc + the host helpers as an executable under a
    host-code sanitizer: kind "address" = ASan + UBSan, "thread" = TSan. GPU
    sanitizers are not available on the MI355X pool; the kernels are covered by the DRN_CHECK_NAN
    and DRN_DETERMINISTIC modes instead."""
    import tempfile
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    san = {"address": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
           "thread": ["-fsanitize=thread"]}[kind]
    out = Path(out_dir or tempfile.mkdtemp(prefix="drn_san_")) / f"host_sanitize_{kind}"
    srcs = sorted(HOST_SRC.glob("*.cc")) + [HOST_SRC / "tests" / "host_sanitize_main.cc"]
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread"] + san + \
        ["-o", str(out)] + [str(s) for s in srcs]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"sanitizer driver build failed:\n{res.stderr[-4000:]}")
    return out


def build_host(force: bool = False, verbose: bool = True) -> Path:
    """Compile the native host helpers (CRC32C, TFRecord scan, CIFAR gather) with g++."""
    srcs = sorted(HOST_SRC.glob("*.cc"))
    newest = max(s.stat().st_mtime for s in srcs)
    if HOST_LIB_PATH.exists() and HOST_LIB_PATH.stat().st_mtime >= newest and not force:
        return HOST_LIB_PATH
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    tmp = HOST_LIB_PATH.with_suffix(".so.tmp")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-o", str(tmp)] + [str(s) for s in srcs]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"host library build failed:\n{res.stderr[-4000:]}")
    os.replace(tmp, HOST_LIB_PATH)
    if verbose:
        print(f"[drn.build] built {HOST_LIB_PATH}")
    return HOST_LIB_PATH


def build(force: bool = False, verbose: bool = True, extra: list[str] | None = None) -> Path:
    """Compile all kernels for gfx950 and link libdrn_kernels.so (incremental)."""
    build_host(force=force, verbose=verbose)
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    if force:
        for o in OBJ_DIR.glob("*.o"):
            o.unlink()
    extra = list(extra or [])
    jobs = min(len(srcs), max(1, min(8, (os.cpu_count() or 4))))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, extra), srcs))
    objs.append(_stamp_object())
    newest = max(o.stat().st_mtime for o in objs)
    if LIB_PATH.exists() and LIB_PATH.stat().st_mtime >= newest and not force:
        if verbose:
            print(f"[drn.build] up to date: {LIB_PATH}")
        return LIB_PATH
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(tmp)] + [str(o) for o in objs]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{res.stderr[-6000:]}")
    os.replace(tmp, LIB_PATH)
    if verbose:
        print(f"[drn.build] built {LIB_PATH} from {len(objs)} translation units for {ARCH}")
    return LIB_PATH


def build_variant(out_dir: str, extra: list[str], src_root: Optional[str] = None) -> Path:
    """A diagnostics / A-B variant of the kernel library (e.g. extra=["-DDRN_CONV_TRACE"]) built
    into out_dir/libdrn_kernels.so with its own objects; load it with DRN_KERNEL_LIB=<path>
    (the source-stamp check is skipped for an explicit library). src_root: a directory holding
    kernels/ and include/ to build instead of csrc/ (patched copies for experiments, e.g.
    scripts/conv_bound_iso.py)."""
    out = Path(out_dir).resolve()
    obj_dir = REPO / "build" / ("variant_" + out.parent.name + "_" + out.name)  # objects stay out of the tree
    out.mkdir(parents=True, exist_ok=True)
    obj_dir.mkdir(parents=True, exist_ok=True)
    kdir = Path(src_root) / "kernels" if src_root else KERNELS
    inc = Path(src_root) / "include" if src_root else INCLUDE
    srcs = sorted(kdir.glob("*.hip"))
    with cf.ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, list(extra), obj_dir, inc), srcs))
    objs.append(_stamp_object())
    lib = out / "libdrn_kernels.so"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib)] + [str(o) for o in objs]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{res.stderr[-6000:]}")
    return lib


if __name__ == "__main__":
    if "--variant" in sys.argv:  # --variant <out_dir> <hipcc flags...>
        i = sys.argv.index("--variant")
        print(build_variant(sys.argv[i + 1], sys.argv[i + 2:]))
    else:
        build(force="--force" in sys.argv)
