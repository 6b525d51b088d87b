"""Test-only: build/load the host emulation of the engine (tests/emu/mt_emu.cpp)."""
import os
import subprocess

from fluidframework_amd.engine import Engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "emu", "mt_emu.cpp")
LIB = os.path.join(ROOT, "tests", "emu", "libmtemu.so")
DEPS = [SRC, os.path.join(ROOT, "include", "mtgpu.h")] + [os.path.join(ROOT, "fluidframework_amd", "csrc", f) for f in
                ("mt_core.h", "mt_replay.h", "mt_snapshot.h", "mt_pack.h", "mt_api_impl.h", "mt_ctx.h", "wave.h", "mt_shard.h",
                 "mt_query.h")]


def _atomic_build(cmd, out):
    """Compile to a private temporary name and rename over `out`, so parallel test
    workers (pytest -n) never load a half-written library."""
    tmp = f"{out}.{os.getpid()}.tmp"
    subprocess.check_call([tmp if a is None else a for a in cmd])
    os.replace(tmp, out)


# MT_EMU_SANITIZE=1: the suite runs on an UndefinedBehaviorSanitizer build of the emulation
# (every UB check aborts the process; tests/emu/sanitize_driver.cpp covers AddressSanitizer)
SANITIZE = os.environ.get("MT_EMU_SANITIZE") == "1"
if SANITIZE:
    LIB = os.path.join(ROOT, "tests", "emu", "libmtemu_ubsan.so")


def build_emu(force=False):
    if force or not os.path.exists(LIB) or any(os.path.getmtime(LIB) < os.path.getmtime(d) for d in DEPS):
        # long-document residency: windows above 64 entries take the multi-wave scan (the device
        # scans up to 512 in wave 0 alone), so the CPU tests' small windows run both paths; every
        # parent-cache hit is checked against the block's parent field (abort on a stale entry)
        san = ["-fsanitize=undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"] if SANITIZE else []
        _atomic_build(["g++", "-O2", "-g", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wno-unknown-pragmas",
                       "-DMT_G_MWMIN=64", "-DMT_BPC_CHECK=1"] + san + ["-o", None, SRC], LIB)
    return LIB


def emu_engine(max_docs, **kw):
    return Engine(max_docs, lib_path=build_emu(), prefix="emu_", **kw)


NAPI_EMU = os.path.join(ROOT, "tests", "emu", "mtgpu_emu_ubsan.node" if SANITIZE else "mtgpu_emu.node")


def build_emu_napi():
    """The product N-API addon source compiled against the host emulation
    (every mt_* call renamed to emu_* by a forced include): lets CPU tests run
    the Node host end to end.  Returns None if Node headers are absent."""
    import re
    if not os.path.exists("/usr/include/node/node_api.h"):
        return None
    lib = build_emu()
    src = os.path.join(ROOT, "fluidframework_amd", "napi", "mtgpu_napi.cpp")
    hdr = os.path.join(ROOT, "include", "mtgpu.h")
    ren = os.path.join(ROOT, "tests", "emu", "emu_rename.h")
    names = sorted(set(re.findall(r"\b(mt_[a-z0-9_]+)\s*\(", open(hdr).read())))
    text = "".join(f"#define {n} emu_{n[3:]}\n" for n in names)
    if not os.path.exists(ren) or open(ren).read() != text:
        tmp = f"{ren}.{os.getpid()}.tmp"
        open(tmp, "w").write(text)
        os.replace(tmp, ren)
    deps = [src, hdr, lib, ren]
    if not os.path.exists(NAPI_EMU) or any(os.path.getmtime(NAPI_EMU) < os.path.getmtime(d) for d in deps):
        _atomic_build(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-I/usr/include/node", "-include", ren,
                       "-o", None, src, lib, "-Wl,-rpath," + os.path.dirname(lib)], NAPI_EMU)
    return NAPI_EMU
