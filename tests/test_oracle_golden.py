"""Pin the oracle against the reference's own golden snapshotV1 fixtures.

The five files under tests/golden/reference_snapshots_v1/ are the reference's
expected outputs (packages/dds/sequence/src/test/snapshots/v1/*.json).  The
recipes below restate generateSharedStrings.ts:23-96 (a detached SharedString
edited by local ops); the oracle must reproduce every blob byte-for-byte.
"""
import json
import os

import pytest

from fluidframework_amd.batch import PropTable
from oracle_lib import OracleDoc

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_snapshots_v1")
# packages/dds/sequence/src/test/snapshots/legacy/*.json (legacyWithCatchUp/*.json are
# byte-identical: these strings are detached, so no catch-up ops are recorded).
GOLD_LEGACY = os.path.join(os.path.dirname(__file__), "golden", "reference_snapshots_legacy")
SIZE_OF_FIRST_CHUNK = 10000  # SnapshotLegacy.sizeOfFirstChunk, snapshotlegacy.ts:57
INSERT_TEXT = "text"


def blobs_of(name, legacy=False):
    d = json.load(open(os.path.join(GOLD_LEGACY if legacy else GOLD, name + ".json")))
    content = [e for e in d["entries"] if e["path"] == "content"][0]["value"]["entries"]
    return {e["path"]: e["value"]["contents"] for e in content}


def build(name):
    s = OracleDoc(collaborating=False, props=PropTable())
    if name == "headerOnly":
        for i in range(int((SIZE_OF_FIRST_CHUNK / len(INSERT_TEXT)) / 2)):
            s.insert_text(0, f"{INSERT_TEXT}{i}")
    elif name in ("headerAndBody", "withMarkers", "withAnnotations"):
        for i in range(int((SIZE_OF_FIRST_CHUNK / len(INSERT_TEXT)) * 2)):
            s.insert_text(0, f"{INSERT_TEXT}{i}")
        if name == "withMarkers":
            i = 0
            while i < s.get_length():
                s.insert_marker(i, 1, {"ItemType": "Paragraph", "Properties": {"Bold": False},
                                       "markerId": f"marker{i}", "referenceTileLabels": ["Eop"]})
                i += 70
        if name == "withAnnotations":
            i = 0
            while i < s.get_length():
                s.annotate_range(i, i + 10, {"bold": True})
                i += 70
    elif name == "largeBody":
        for i in range(SIZE_OF_FIRST_CHUNK):
            s.insert_text(0, f"{INSERT_TEXT}-{i}")
    return s


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"])
def test_oracle_reproduces_reference_snapshot(name):
    want = blobs_of(name)
    s = build(name)
    blobs, _ = s.snapshot(0, 0)
    got = {("header" if i == 0 else f"body_{i - 1}"): b.decode("utf-8") for i, b in enumerate(blobs)}
    assert list(got) == list(want)
    for k in want:
        assert got[k] == want[k], f"{name}/{k} differs"


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"])
def test_oracle_reproduces_reference_legacy_snapshot(name):
    """SnapshotLegacy (the default format, snapshotlegacy.ts:104-240): header and body."""
    want = blobs_of(name, legacy=True)
    s = build(name)
    blobs, _ = s.snapshot(0, 0, legacy=True)
    got = {("header" if i == 0 else "body"): b.decode("utf-8") for i, b in enumerate(blobs)}
    assert list(got) == list(want)
    for k in want:
        assert got[k] == want[k], f"legacy/{name}/{k} differs"
