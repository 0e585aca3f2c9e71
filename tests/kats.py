"""Loader for tests/golden/reference_kats.json (the reference's own KATs)."""
import json
import os

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_kats.json")


def load():
    with open(PATH) as fh:
        vecs = json.load(fh)["vectors"]
    for v in vecs:
        v["data"] = bytes.fromhex(v.get("data", ""))
    return vecs


def by_kind(*kinds):
    return [v for v in load() if v["kind"] in kinds]
