"""In-tree build of libvp3d.so (the C-ABI of include/vp3d.h) for gfx950.

Plain `hipcc` per translation unit, then one shared-library link.  An object is
rebuilt only when its own source, or the shared configuration (target arch, flags,
any header, this recipe), changed -- by content hash, recorded beside the object --
so editing one kernel recompiles one file.  The library lands next to this file so
that it travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_PKG = os.path.dirname(PKG_DIR)                       # dynamic-camera-augmented-videopose3d_amd/
REPO = os.path.dirname(ROOT_PKG)
CSRC = os.path.join(ROOT_PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
BUILD_DIR = os.path.join(ROOT_PKG, "build")
LIB_PATH = os.path.join(PKG_DIR, "libvp3d.so")

SOURCES = ["conv_gemm.hip", "conv_gemm_big.hip", "conv_gemm_8p.hip", "conv_gemm_q64.hip", "conv_gemm_a4.hip", "conv_gemm_tail.hip", "expand_gemm.hip", "preprocess.hip",
           "metrics.hip", "stream_step.hip", "stream_persist.hip", "stream_pipe.hip", "train.hip", "seq_lifter.hip", "vp3d_capi.cpp", "vp3d_train.cpp",
           "vp3d_seq.cpp"]
ARCH = os.environ.get("VP3D_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: HIP defaults to fast contraction, and the HIP headers' __fmul_rn /
# __fadd_rn carry that flag from their own definition, so a per-file pragma is not
# enough to keep the reference's separately rounded mul/add sequences intact.
COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-I", INCLUDE, "-I", CSRC,
                "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-value",
                "-Wno-unused-result"]


def _hashed_files():
    """Every file the library is built from: the translation units, every header under
    csrc/ and include/, and this build recipe itself."""
    files = [os.path.join(CSRC, s) for s in SOURCES]
    for d in (CSRC, INCLUDE):
        files += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp")))
    files.append(os.path.abspath(__file__))
    return files


def source_hash() -> str:
    """SHA-256 over (relative path, contents) of the sources, the target arch and the
    compiler flags: the provenance string embedded in libvp3d.so (vp3d_build_hash)."""
    import hashlib
    h = hashlib.sha256()
    h.update(("arch=" + ARCH + ";flags=" + " ".join(COMMON_FLAGS[:4] + COMMON_FLAGS[8:])).encode())
    for f in _hashed_files():
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def embedded_hash(path: str = LIB_PATH):
    """The source hash a built library carries (read from the file, without loading it)."""
    import re
    try:
        with open(path, "rb") as f:
            m = re.search(rb"VP3D_SRC_SHA256=([0-9a-f]{64})", f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _config_hash() -> str:
    """Hash of what every object depends on besides its own source: arch, flags, the
    headers under csrc/ and include/, and this recipe."""
    import hashlib
    h = hashlib.sha256(("arch=" + ARCH + ";flags=" + " ".join(COMMON_FLAGS)).encode())
    for f in _hashed_files()[len(SOURCES):]:
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _tu_hash(config: str, src: str) -> str:
    import hashlib
    h = hashlib.sha256(config.encode())
    with open(src, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()


def _stale(obj: str, tu: str) -> bool:
    try:
        with open(obj + ".sha") as f:
            return f.read().strip() != tu or not os.path.exists(obj)
    except OSError:
        return True


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n$ " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


LLVM_BIN = os.environ.get("VP3D_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
# kernels that own the accumulator file through inline asm (named AGPRs, no clobbers per
# MFMA): the compiler must never place a value of its own in an AGPR there
AGPR_OWNERS = ("conv_gemm_a4.hip",)


def agpr_writes(obj: str) -> int:
    """v_accvgpr_write instructions in the gfx950 code object of a compiled translation unit.
    In conv_gemm_a4 every AGPR holds an accumulator the MFMAs write through inline asm, so a
    v_accvgpr_write there is the register allocator spilling a VGPR into the accumulator file
    (it happens once the kernel needs more than 256 VGPRs) -- silently wrong results."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fatbin"), os.path.join(d, "dev.co")
        _run([os.path.join(LLVM_BIN, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x.o")])
        _run([os.path.join(LLVM_BIN, "clang-offload-bundler"), "--type=o", f"--input={fb}",
              f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--output={co}", "--unbundle"])
        dis = _run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", co])
    return dis.count("v_accvgpr_write")


def build(verbose: bool = False, force: bool = False, jobs: int | None = None) -> str:
    """Compile every stale translation unit (in parallel: hipcc is single-threaded
    per file) and link libvp3d.so."""
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(BUILD_DIR, exist_ok=True)
    want = source_hash()
    config = _config_hash()
    objs, todo = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        if not os.path.exists(src):
            continue
        obj = os.path.join(BUILD_DIR, s + ".o")
        objs.append(obj)
        tu = _tu_hash(config, src)
        if force or _stale(obj, tu):
            if s.endswith(".hip"):
                cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}"] + COMMON_FLAGS + ["-c", src, "-o", obj]
            else:
                cmd = [HIPCC] + COMMON_FLAGS + ["-c", src, "-o", obj]
            todo.append((cmd, obj, tu))
    if todo:
        jobs = jobs or max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
        for cmd, obj, _ in todo:
            if verbose:
                print("$", " ".join(cmd), flush=True)
            if os.path.exists(obj + ".sha"):
                os.remove(obj + ".sha")
        with ThreadPoolExecutor(jobs) as ex:
            for out in ex.map(_run, [t[0] for t in todo]):
                if verbose and out.strip():
                    print(out)
        for _, obj, tu in todo:
            if os.path.basename(obj)[:-2] in AGPR_OWNERS:
                n = agpr_writes(obj)
                if n:
                    os.remove(obj)
                    raise RuntimeError(f"build failed: {os.path.basename(obj)} spills {n} values into the "
                                       "accumulator registers (v_accvgpr_write): cut VGPR pressure")
            with open(obj + ".sha", "w") as f:
                f.write(tu + "\n")
    if force or todo or embedded_hash() != want:
        # provenance: one generated translation unit carrying the source hash
        info_src = os.path.join(BUILD_DIR, "build_info.cpp")
        info_obj = info_src + ".o"
        with open(info_src, "w") as f:
            f.write('// generated by vp3d_amd/build.py\n'
                    f'static const char kTag[] = "VP3D_SRC_SHA256={want}";\n'
                    'extern "C" const char* vp3d_build_hash(void) { return kTag + 16; }\n')
        _run([HIPCC] + COMMON_FLAGS + ["-c", info_src, "-o", info_obj])
        objs.append(info_obj)
        # -z defs: an unresolved symbol (e.g. a kernel launch stub the host compilation dropped)
        # fails the link here instead of the library load on the GPU box
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-Wl,-z,defs", "-o", LIB_PATH] + objs
        if verbose:
            print("$", " ".join(cmd), flush=True)
        _run(cmd)
    return LIB_PATH


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
