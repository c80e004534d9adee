"""Build the in-tree native libraries.

* ``libdcrt.so``  -- the product: host scene/BVH/loader C++ and the gfx950 HIP
  kernels + tracer, one shared object behind the C ABI of ``include/dcrt.h``.
* ``oracle/build/libdcrt_oracle.so`` -- the CPU restatement used only by tests
  and the bench's ``cpu_baseline`` leg (test infrastructure, never the product).

Both compile with IEEE single precision and no floating-point contraction so the
GPU path and the oracle produce the same bits ("Numerics").
"""
from __future__ import annotations

import contextlib
import fcntl
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
LIB_PATH = PKG_DIR / "libdcrt.so"
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "build" / "libdcrt_oracle.so"

HOST_SOURCES = sorted((CSRC / "host").glob("*.cpp"))
DEVICE_SOURCES = [CSRC / "device" / "tracer.hip"]
HEADERS = sorted((CSRC / "host").glob("*.h")) + sorted((CSRC / "device").glob("*.h")) + [ROOT / "include" / "dcrt.h"]

HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=off",      # no FMA contraction: bit-identical to the oracle
    "-fno-fast-math",
    # no SLP vectorisation: its packed-f32 ops (v_pk_mul/add_f32, same IEEE results) cost
    # registers (cast kernel 96 -> 78 VGPRs, MATERIAL 117 -> 104, 152 -> 125 without) and
    # pair the refill's prefetch register with operands that then wait for it: Cornell
    # 1080p 3.75 -> 3.49 ms/spp (tools/ab_libs.sh, two passes)
    "-fno-slp-vectorize",
    "-fno-gpu-rdc",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
    "-Wno-unused-but-set-variable",
]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MI355X build needs ROCm's hipcc")


def _digest(paths) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(str(p).encode())
        h.update(Path(p).read_bytes())
    h.update(" ".join(HIPCC_FLAGS).encode())
    return h.hexdigest()


@contextlib.contextmanager
def _build_lock(name: str):
    """One build of an output at a time across processes (pytest-xdist workers, a test and a
    tool): its object directory and stamp are shared, and two compilers writing one object
    file leave a corrupt library. Different outputs build concurrently."""
    PKG_DIR.mkdir(exist_ok=True)
    with open(PKG_DIR / f".build.{name}.lock", "w") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)


def _fresh(lib: Path, stamp: Path, digest: str) -> bool:
    return lib.exists() and stamp.exists() and stamp.read_text().strip() == digest


def build_native(force: bool = False, verbose: bool = False, out: Path | None = None, extra_flags=()) -> Path:
    """Compile libdcrt.so (or an experimental variant at `out` with `extra_flags`)."""
    lib_path = Path(out) if out else LIB_PATH
    sources = HOST_SOURCES + DEVICE_SOURCES
    digest = _digest(sources + HEADERS) + " ".join(extra_flags)
    stamp = lib_path.with_suffix(".so.sha256")
    if not force and _fresh(lib_path, stamp, digest):
        return lib_path
    with _build_lock(lib_path.stem):
        if not force and _fresh(lib_path, stamp, digest):   # (another process built it meanwhile)
            return lib_path
        return _build_native_locked(lib_path, stamp, digest, out, verbose, extra_flags)


def _build_native_locked(lib_path: Path, stamp: Path, digest: str, out, verbose: bool, extra_flags) -> Path:
    sources = HOST_SOURCES + DEVICE_SOURCES
    objdir = PKG_DIR / ("_build" if out is None else "_build_" + lib_path.stem)
    objdir.mkdir(exist_ok=True)
    objs = []
    procs = []
    for src in sources:
        obj = objdir / (src.stem + (".dev.o" if src.suffix == ".hip" else ".o"))
        cmd = [_hipcc(), *HIPCC_FLAGS, *extra_flags, "-c", str(src), "-o", str(obj)]
        if src.suffix == ".cpp":
            cmd = [_hipcc(), *[f for f in HIPCC_FLAGS if f not in ("--offload-arch=gfx950", "-fno-gpu-rdc")],
                   "-x", "c++", "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    failed = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((src, out.decode(errors="replace")))
        elif verbose and out:
            print(out.decode(errors="replace"), file=sys.stderr)
    if failed:
        msg = "\n".join(f"--- {s} ---\n{o}" for s, o in failed)
        raise RuntimeError(f"native build failed:\n{msg}")
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib_path)
    stamp.write_text(digest)
    return lib_path


SANITIZED_LIB = PKG_DIR / "_build_asan" / "libdcrt_asan.so"


def build_sanitized(force: bool = False) -> Path:
    """TEST TOOLING: libdcrt.so with the host code under AddressSanitizer + UBSan (the OBJ / XML
    parsers, the BVH builder, the scene and C-ABI code; the tracer's host side through
    -Xarch_host, the device code unchanged). tools/sanitize_host.sh runs the CPU suite against
    it (DCRT_LIB) with clang's ASan runtime preloaded."""
    san = ["-fsanitize=address", "-fsanitize=undefined"]
    sources = HOST_SOURCES + DEVICE_SOURCES
    digest = _digest(sources + HEADERS) + "asan"
    stamp = SANITIZED_LIB.with_suffix(".so.sha256")
    if not force and _fresh(SANITIZED_LIB, stamp, digest):
        return SANITIZED_LIB
    with _build_lock("asan"):
        if not force and _fresh(SANITIZED_LIB, stamp, digest):
            return SANITIZED_LIB
        return _build_sanitized_locked(san, sources, stamp, digest)


def _build_sanitized_locked(san, sources, stamp: Path, digest: str) -> Path:
    objdir = SANITIZED_LIB.parent
    objdir.mkdir(exist_ok=True)
    objs, procs = [], []
    for src in sources:
        obj = objdir / (src.stem + (".dev.o" if src.suffix == ".hip" else ".o"))
        if src.suffix == ".cpp":
            cmd = [_hipcc(), *[f for f in HIPCC_FLAGS if f not in ("--offload-arch=gfx950", "-fno-gpu-rdc", "-O3")], "-O1", "-g",
                   "-fno-omit-frame-pointer", *san, "-x", "c++", "-c", str(src), "-o", str(obj)]
        else:
            cmd = [_hipcc(), *HIPCC_FLAGS, "-g", *[x for f in san for x in ("-Xarch_host", f)], "-c", str(src), "-o", str(obj)]
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"sanitized build failed: {src}\n{out.decode(errors='replace')}")
    subprocess.run([_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *san, "-shared-libasan", "-o", str(SANITIZED_LIB),
                    *map(str, objs)], check=True)
    stamp.write_text(digest)
    return SANITIZED_LIB


EXAMPLE_SRC = ROOT / "examples" / "dcrt_render.cpp"
EXAMPLE_SOURCES = [EXAMPLE_SRC, ROOT / "examples" / "mi355x_path_tracer.cpp"]
EXAMPLE_HEADERS = [ROOT / "examples" / "mi355x_path_tracer.h", ROOT / "examples" / "renderer_loop.h"]
EXAMPLE_BIN = ROOT / "examples" / "dcrt_render"


def build_examples(force: bool = False) -> Path:
    """examples/dcrt_render: a C++ host of libdcrt.so through the C ABI alone -- the reference's
    CPathTracer plugin slot filled by CMI355XPathTracer, driven by its frame loop."""
    lib = build_native()
    digest = _digest([*EXAMPLE_SOURCES, *EXAMPLE_HEADERS, ROOT / "include" / "dcrt.h", lib])
    stamp = EXAMPLE_BIN.with_suffix(".sha256")
    if not force and _fresh(EXAMPLE_BIN, stamp, digest):
        return EXAMPLE_BIN
    with _build_lock("examples"):
        if not force and _fresh(EXAMPLE_BIN, stamp, digest):
            return EXAMPLE_BIN
        cxx = shutil.which("g++") or "g++"
        cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-Wextra", *map(str, EXAMPLE_SOURCES), "-I", str(ROOT / "include"),
               "-L", str(PKG_DIR), "-ldcrt",
               "-Wl,-rpath,$ORIGIN/../directcomputeraytracing_amd", "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(EXAMPLE_BIN)]
        subprocess.run(cmd, check=True)
        stamp.write_text(digest)
    return EXAMPLE_BIN


def build_oracle(force: bool = False) -> Path:
    """TEST INFRASTRUCTURE: compile the CPU restatement (gcc, no contraction)."""
    src = [ORACLE_DIR / "dcrt_oracle.c", ORACLE_DIR / "dcrt_oracle_bvh.c", ORACLE_DIR / "dcrt_oracle_scene.c",
           ORACLE_DIR / "dcrt_oracle.h",
           ORACLE_DIR / "Makefile", ROOT / "include" / "dcrt.h"]
    digest = _digest(src)
    stamp = ORACLE_LIB.with_suffix(".so.sha256")
    if not force and _fresh(ORACLE_LIB, stamp, digest):
        return ORACLE_LIB
    with _build_lock("oracle"):
        if not force and _fresh(ORACLE_LIB, stamp, digest):
            return ORACLE_LIB
        subprocess.run(["make", "-C", str(ORACLE_DIR), f"OUT={ORACLE_LIB.parent}"], check=True,
                       stdout=subprocess.DEVNULL)
        stamp.write_text(digest)
    return ORACLE_LIB


REFERENCE = Path(os.environ.get("DCRT_REFERENCE", "/root/reference"))


def build_reference_checkers() -> Path | None:
    """TEST INFRASTRUCTURE: when the reference sources are present (the build container,
    never the GPU box), compile its own OBJ dependencies -- tinyobjloader + MikkTSpace,
    unmodified, from where they lie -- with our load-flow harness into
    oracle/_ref/librefobj.so (oracle/ref_obj/Makefile). tests/test_obj_pin.py uses it."""
    if not (REFERENCE / "tinyobjloader" / "tiny_obj_loader.h").exists():
        return None
    with _build_lock("reference"):
        subprocess.run(["make", "-s", "-C", str(ORACLE_DIR / "ref_obj"), f"REF={REFERENCE}"], check=True,
                       stdout=subprocess.DEVNULL)
        # ... and its vendored RapidXml for tests/test_xml_pin.py (oracle/ref_xml/Makefile)
        if (REFERENCE / "RapidXml" / "rapidxml.hpp").exists():
            subprocess.run(["make", "-s", "-C", str(ORACLE_DIR / "ref_xml"), f"REF={REFERENCE}"], check=True,
                           stdout=subprocess.DEVNULL)
    return ORACLE_DIR / "_ref" / "librefobj.so"


if __name__ == "__main__":
    print(build_native(force="--force" in sys.argv, verbose=True))
    print(build_oracle(force="--force" in sys.argv))
    print(build_examples(force="--force" in sys.argv))
