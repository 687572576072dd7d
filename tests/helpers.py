"""Shared helpers for the test suite."""
import json
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def config(name):
    with open(os.path.join(ROOT, "configs", f"{name}.yml")) as f:
        return yaml.safe_load(f)


def reference_doc(name):
    with open(os.path.join(GOLDEN, "reference_data", name)) as f:
        return f.read()


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def diff_verdicts(gpu, ora, npol, ids, limit=8):
    """Human-readable first mismatches between two verdict arrays."""
    import kwgpu as K
    bad = (gpu != ora).nonzero()[0]
    lines = []
    for i in bad[:limit]:
        r, j = divmod(int(i), npol)
        lines.append(f"row {r} policy {ids[j]}: gpu {K.decode(gpu[i])} oracle {K.decode(ora[i])}")
    return f"{len(bad)} mismatches\n" + "\n".join(lines)
