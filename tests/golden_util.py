"""Helpers to read the committed golden fixtures (tests/golden/)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def reference_vectors():
    with open(os.path.join(GOLDEN, "reference_vectors.json")) as f:
        return json.load(f)


def xxh3_vectors():
    with open(os.path.join(GOLDEN, "xxh3_vectors.json")) as f:
        meta = json.load(f)
    blob = np.fromfile(os.path.join(GOLDEN, "xxh3_vectors.bin"), dtype=np.uint8)
    return blob, meta["vectors"]


def batch_cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        c["data"] = np.fromfile(os.path.join(GOLDEN, c["file"]), dtype=np.uint8)
    return cases


def expect_matches(expect: dict, err) -> bool:
    if expect["kind"] != err.kind:
        return False
    for k in ("reason", "a", "b", "c"):
        if k in expect and expect[k] != getattr(err, k):
            return False
    return True
