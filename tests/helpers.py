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


def wide_docs():
    """70 Pod reviews, some with more than 64 containers / labels (entity indices past one byte of
    the reason argument): added / dropped capabilities, AppArmor annotations, C4 label keys."""
    caps = ["NET_ADMIN", "SYS_TIME", "CHOWN", "KILL", "SETUID", "MKNOD"]
    keys = ["app", "tier", "env", "team", "owner", "version", "legacy", "debug", "region", "pci"]
    docs = []
    for r in range(70):
        n_ctr = 80 if r % 9 == 0 else 1 + r % 3
        n_lbl = 90 if r % 11 == 0 else r % 5
        ctrs = [{"name": f"c{i}", "image": "nginx",
                 "securityContext": {"capabilities": {"add": [caps[(i + j + r) % 6] for j in range((i + r) % 3)],
                                                      "drop": ["KILL"] if (i + r) % 4 == 0 else []}}}
                for i in range(n_ctr)]
        labels = {(keys[i % len(keys)] if i < len(keys) else f"k{i}"): ("v%d" % i if i % 3 else "x" * (i % 7))
                  for i in range(n_lbl)}
        meta = {"labels": labels}
        if r % 2:
            meta["annotations"] = {f"container.apparmor.security.beta.kubernetes.io/c{i}": "runtime/default"
                                   for i in range(0, n_ctr, 2)}
        docs.append({"request": {"uid": str(r), "kind": {"group": "", "version": "v1", "kind": "Pod"},
                                 "resource": {"group": "", "version": "v1", "resource": "pods"},
                                 "operation": "CREATE", "userInfo": {},
                                 "object": {"kind": "Pod", "metadata": meta, "spec": {"containers": ctrs}}}})
    return docs
