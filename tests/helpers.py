"""Shared helpers for the test suite."""
import json
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def config(name):
    with open(os.path.join(ROOT, "configs", f"{name}.yml")) as f:
        return yaml.safe_load(f)


def many_policies_config():
    """configs/c6_256.yml: 256 policies whose request columns hold hundreds of patterns each and a
    40-member group (synth config 6 draws from the same vocabularies)."""
    return config("c6_256")


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


def wide_entity_case():
    """(AdmissionReview, policies): 300 containers and 300 labels; container c299 adds NET_ADMIN
    (every other container adds only allowed CHOWN), container c270 runs AppArmor profile
    localhost/evil, label k299 has value 'bad' against the constraint '^ok$' (every other label's
    value is 'ok'), and label k280 is denied (VERDICT r01 "What's weak" #1 repro, extended)."""
    ctrs = [{"name": f"c{i}", "image": "ghcr.io/x/y:1.0",
             "securityContext": {"capabilities": {"add": ["NET_ADMIN"] if i == 299 else ["CHOWN"]}}}
            for i in range(300)]
    labels = {f"k{i}": ("bad" if i == 299 else "ok") for i in range(300)}
    ann = {f"container.apparmor.security.beta.kubernetes.io/c{i}": ("localhost/evil" if i == 270 else "runtime/default")
           for i in range(300)}
    doc = {"request": {"uid": "wide", "kind": {"group": "", "version": "v1", "kind": "Pod"},
                       "resource": {"group": "", "version": "v1", "resource": "pods"}, "operation": "CREATE",
                       "userInfo": {}, "object": {"kind": "Pod", "metadata": {"labels": labels, "annotations": ann},
                                                  "spec": {"containers": ctrs}}}}
    mod = "registry://ghcr.io/kubewarden/policies/"
    pols = {
        "caps": {"module": mod + "psp-capabilities:v0.1.7", "settings": {"allowed_capabilities": ["CHOWN"]}},
        "labels": {"module": mod + "safe-labels:v0.1.14", "settings": {"constrained_labels": {"k299": "^ok$", "k5": "^ok$"}}},
        "labels-denied": {"module": mod + "safe-labels:v0.1.14", "settings": {"denied_labels": ["k280", "k290"]}},
        "apparmor": {"module": mod + "psp-apparmor:v0.1.7", "settings": {"allowed_profiles": ["runtime/default"]}},
    }
    return json.dumps(doc), pols
