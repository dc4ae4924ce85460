"""Test frames shared by the CPU and GPU suites (test infrastructure)."""
import importlib.util
import os
import random

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def golden_twin():
    """tests/golden/make_golden.py, the independent Python restatement of the wire rules."""
    spec = importlib.util.spec_from_file_location("mg", os.path.join(HERE, "golden",
                                                                     "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def rich_wire(n, seed, corrupt_at=None):
    """A frame the byte-range decoders decline: every Value tag with Maps, nested arrays and
    Error(Value) (the golden twin's generator), Heartbeats and Unsubscribed messages, ids past
    35 bits. corrupt_at: the message index replaced by an Update with an unknown value tag."""
    mg = golden_twin()
    rng = random.Random(seed)
    msgs = []
    for _ in range(n):
        k = rng.random()
        if k < 0.04:
            msgs.append(("hb",))
        elif k < 0.06:
            msgs.append(("raw", 2, mg.enc_varint(rng.getrandbits(20))))
        else:
            msgs.append(("u", rng.getrandbits(rng.choice([7, 14, 30, 40])), mg.rand_value(rng)))
    if corrupt_at is not None:
        msgs[corrupt_at] = ("raw", 4, mg.enc_varint(5) + bytes([77]))  # Update, value tag 77
    wire, _ = mg.batch(msgs)
    return np.frombuffer(wire, np.uint8).copy()
