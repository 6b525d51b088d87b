"""Whole-population parity at the bench configurations' full sizes, on the GPU: bench.py replays
configs 3, 4 and 5 exactly as its measurement does (every document of the workload, the same
seeds) and every document's SnapshotV1 digest must equal the oracle-made manifest
(tests/golden/digests, tools/make_digest_manifest.py: the oracle's own generator and replay).
Config 2's is checked by the default bench line itself.  These run in the -m gpu suite so the
round-end GPU tier checks configs 3-5 at full size, not only down-scaled."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    "config3": 16384,          # 16,384 docs x 4,000 msgs, annotate-heavy, zamboni
    "config4": 256,            # 256 docs pre-built to 200k segments, 50k msgs each
    "config5": 131072,         # 131,072 Zipf-sized docs through the LPT exchange path
}


def bench_line(cfg: str) -> dict:
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--no-ingest"], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", sorted(CASES))
def test_full_scale_manifest_parity_on_gpu(cfg):
    out = bench_line(cfg)
    man = out.get("parity_manifest")
    assert man is not None, out["parity"]
    assert man["checked"] == man["of"] == CASES[cfg], man
    assert man["mismatches"] == 0, man
    assert "STATUS ERROR" not in out["parity"] and "MISMATCH" not in out["parity"], out["parity"]
