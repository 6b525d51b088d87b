"""Oracle known-answer tests restated from the reference's own merge-tree specs.

* MT/test/mergeTree.markRangeRemoved.spec.ts:59-100 (remote remove/insert races)
* MT/test/client.applyMsg.spec.ts:23-88 (100 interleaved ops from one client:
  a passive observer must end with the author's text)
* MergeTree.insertingWalk.spec.ts:187-253 (insert at beginning/end/middle of
  trees of several shapes) -- restated as single-author streams whose observer
  text must equal a plain string model.
"""
import random

import numpy as np

from fluidframework_amd.batch import BatchBuilder, ClientNames, PropTable
from oracle_lib import OracleDoc


def run_msgs(msgs, props=None):
    props = props or PropTable()
    names = ClientNames()
    bb = BatchBuilder(props, names)
    bb.begin_doc(0)
    for m in msgs:
        bb.add_message(m)
    batch = bb.build()
    d = OracleDoc(True, props, names.json_literals())
    st = d.apply_run(batch, 0)
    return d, st


def msg(client, seq, ref, op, msn=0):
    return dict(clientId=client, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn,
                type="op", contents=op)


def hello_world():
    out = []
    for i, ch in enumerate("hello world"):
        out.append(msg("local", i + 1, i, {"type": 0, "pos1": i, "seg": ch}))
    return out


def test_remote_remove_followed_by_remote_insert():
    m = hello_world()
    m.append(msg("remote2", 12, 11, {"type": 1, "pos1": 0, "pos2": 11}))
    m.append(msg("remote", 13, 11, {"type": 0, "pos1": 0, "seg": "text"}))
    d, st = run_msgs(m)
    assert st == 0 and d.get_text() == "text"


def test_remote_insert_followed_by_remote_remove():
    m = hello_world()
    m.append(msg("remote", 12, 11, {"type": 0, "pos1": 0, "seg": "text"}))
    m.append(msg("remote2", 13, 11, {"type": 1, "pos1": 0, "pos2": 11}))
    d, st = run_msgs(m)
    assert st == 0 and d.get_text() == "text"


def test_interleaved_single_client_ops_match_author():
    # client.applyMsg.spec.ts:23-88: positions computed on the author's view.
    text = "hello world"
    m = [msg("localUser", 1, 0, {"type": 0, "pos1": 0, "seg": text})]
    for i in range(100):
        ln = len(text)
        pos1 = ln // 2
        imod6 = i % 6
        if imod6 in (0, 5):
            pos2 = max((ln - pos1) // 4 - imod6 + pos1, pos1 + 1)
            m.append(msg("localUser", i + 2, 0, {"type": 1, "pos1": pos1, "pos2": pos2}))
            text = text[:pos1] + text[pos2:]
        elif imod6 in (1, 4):
            s = f"{i}" * (imod6 + 5)
            m.append(msg("localUser", i + 2, 0, {"type": 0, "pos1": pos1, "seg": s}))
            text = text[:pos1] + s + text[pos1:]
        else:
            pos2 = max((ln - pos1) // 3 - imod6 + pos1, pos1 + 1)
            m.append(msg("localUser", i + 2, 0, {"type": 2, "pos1": pos1, "pos2": pos2, "props": {"foo": f"{i}"}}))
    d, st = run_msgs(m)
    assert st == 0
    assert d.get_text() == text


def test_single_author_random_streams_match_string_model():
    rng = random.Random(1234)
    for trial in range(20):
        text, msgs, seq = "", [], 0
        lag_author = trial % 2 == 0  # refSeq lagging: still sees own ops
        for _ in range(400):
            ln = len(text)
            seq += 1
            ref = max(0, seq - 1 - (rng.randint(0, 5) if lag_author else 0))
            r = rng.random()
            if ln == 0 or r < 0.5:
                p = rng.randint(0, ln)
                s = "".join(rng.choice("abcdefgh\n") for _ in range(rng.randint(1, 6)))
                msgs.append(msg("A", seq, ref, {"type": 0, "pos1": p, "seg": s}, msn=0))
                text = text[:p] + s + text[p:]
            elif r < 0.8:
                a = rng.randint(0, ln - 1)
                b = min(ln, a + rng.randint(1, 8))
                msgs.append(msg("A", seq, ref, {"type": 1, "pos1": a, "pos2": b}, msn=0))
                text = text[:a] + text[b:]
            else:
                a = rng.randint(0, ln - 1)
                b = min(ln, a + rng.randint(1, 8))
                msgs.append(msg("A", seq, ref, {"type": 2, "pos1": a, "pos2": b, "props": {"k": rng.randint(0, 2)}}, msn=0))
        d, st = run_msgs(msgs)
        assert st == 0
        assert d.get_text() == text, trial
        assert d.get_length() == len(text)


def test_concurrent_insert_tie_break_newer_first():
    # breakTie (mergeTree.ts:2287-2290): a remote insert at the position of a
    # concurrent (unseen) insert goes BEFORE it ("newer segments come first").
    m = [msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "xy"}),
         msg("B", 2, 1, {"type": 0, "pos1": 1, "seg": "1"}),
         msg("C", 3, 1, {"type": 0, "pos1": 1, "seg": "2"})]
    d, _ = run_msgs(m)
    assert d.get_text() == "x21y"
