"""TEST-ONLY driver: runs bench.py's code paths (launcher, per-rank replay, barrier +
max-over-ranks timing, config 5's LPT redistribution and digest gather, the digest
parity check) on the host emulation of the engine with gloo, so the multi-rank logic is
covered on CPU.  Its numbers are emulation timings, never a measurement."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
from emu_lib import build_emu  # noqa: E402
from fluidframework_amd.engine import Engine  # noqa: E402

LIB = build_emu()
bench.Host.factory = staticmethod(lambda n, device=0, **kw: Engine(n, lib_path=LIB, prefix="emu_", **kw))
bench.Host.backend = "gloo"
bench.Host.device_type = "cpu"

if __name__ == "__main__":
    bench.main(sys.argv[1:])
