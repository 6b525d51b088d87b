"""Test-only helpers for the Node host: turn generated op batches back into
ISequencedDocumentMessage lists and run tests/js/replay_check.js on them."""
import json
import os
import shutil
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "js", "replay_check.js")
NODE = shutil.which("node")


def batch_to_messages(batch, props, run):
    """Messages (protocol.ts:126-166) of one document run; client i is "c{i}"."""
    a = batch.arrays
    sets = []
    for s in props.sets:
        sets.append({props.keys[k]: (None if v < 0 else json.loads(props.values_json[v])) for k, v in s})
    out = []
    for i in range(int(batch.op_offsets[run]), int(batch.op_offsets[run + 1])):
        t, fl = int(a["type"][i]), int(a["flags"][i])
        m = dict(clientId=f"c{int(a['client'][i])}", sequenceNumber=int(a["seq"][i]),
                 referenceSequenceNumber=int(a["ref_seq"][i]), minimumSequenceNumber=int(a["msn"][i]), type="op")
        if t == 0:
            o, n = int(a["payload_off"][i]), int(a["payload_len"][i])
            text = bytes(np.asarray(batch.payload[o:o + n], np.uint16).tobytes()).decode("utf-16-le")
            m["contents"] = {"type": 0, "pos1": int(a["pos1"][i]), "seg": text}
        elif t == 1:
            m["contents"] = {"type": 1, "pos1": int(a["pos1"][i]), "pos2": int(a["pos2"][i])}
        elif t == 2:
            c = {"type": 2, "pos1": int(a["pos1"][i]), "pos2": int(a["pos2"][i]), "props": sets[int(a["prop_id"][i])]}
            if fl & 4:
                c["combiningOp"] = {"name": "rewrite"}
            m["contents"] = c
        else:
            m["type"] = "noop"
            m["contents"] = None
        assert fl & 1, "generated streams have one member per message"
        out.append(m)
    return out


def run_driver(name, spec, addon=None, timeout=240):
    """Run tests/js/<name> on a JSON spec; returns its JSON output."""
    env = dict(os.environ)
    if addon:
        env["MTGPU_NAPI"] = addon
    with tempfile.TemporaryDirectory() as td:
        ip, op = os.path.join(td, "in.json"), os.path.join(td, "out.json")
        json.dump(spec, open(ip, "w"))
        subprocess.run([NODE, os.path.join(ROOT, "tests", "js", name), ip, op], check=True, env=env, timeout=timeout)
        return json.load(open(op))


def run_node(doc_msgs, addon=None, limits=None, timeout=240, loads=None, legacy=None, queries=None, options=None):
    env = dict(os.environ)
    if addon:
        env["MTGPU_NAPI"] = addon
    with tempfile.TemporaryDirectory() as td:
        ip, op = os.path.join(td, "in.json"), os.path.join(td, "out.json")
        spec = {"docs": doc_msgs, "limits": limits or {}, "loads": loads, "legacy": legacy, "queries": queries}
        if options is not None:
            spec["options"] = options            # the Clients' options (newClient(options))
        json.dump(spec, open(ip, "w"))
        subprocess.run([NODE, DRIVER, ip, op], check=True, env=env, timeout=timeout)
        return json.load(open(op))
