"""Test-only: build/load the host emulation of the engine (tests/emu/mt_emu.cpp)."""
import os
import subprocess

from fluidframework_amd.engine import Engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "emu", "mt_emu.cpp")
LIB = os.path.join(ROOT, "tests", "emu", "libmtemu.so")
DEPS = [SRC] + [os.path.join(ROOT, "fluidframework_amd", "csrc", f) for f in
                ("mt_core.h", "mt_replay.h", "mt_snapshot.h", "mt_api_impl.h", "mt_ctx.h", "wave.h")]


def build_emu(force=False):
    if force or not os.path.exists(LIB) or any(os.path.getmtime(LIB) < os.path.getmtime(d) for d in DEPS):
        subprocess.check_call(["g++", "-O2", "-g", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                               "-o", LIB, SRC])
    return LIB


def emu_engine(max_docs, **kw):
    return Engine(max_docs, lib_path=build_emu(), prefix="emu_", **kw)
