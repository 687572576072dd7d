"""CPU: the flattener (kw_batch_from_json) against the oracle's independent restatement of the
extraction rules (oracle.flatten_doc, from Python's own JSON reader) on randomly shaped documents:
every workload kind and an unknown one, missing or mistyped members at each level (spec as a list,
containers as an object, numeric names, null images, "true" as a string, capability lists with
non-strings, numeric label values), AppArmor annotations on the pod or the template, escaped and
non-ASCII strings, duplicate keys, raw reviews. Rows must be identical, and a body the oracle
rejects must be rejected by the product (and the other way round)."""
import json
import random

import numpy as np
import pytest

import kwgpu as K
import oracle as O

KINDS = ["Pod", "Deployment", "ReplicaSet", "StatefulSet", "DaemonSet", "Job", "ReplicationController", "CronJob",
         "Namespace", "Service", None]
NAMES = ["web", "db", "sidecar", "cé", "a\"b", "x/y", "", "long-" + "n" * 40]
IMAGES = ["nginx", "ghcr.io/org/app:1.2", "quay.io/a/b@sha256:" + "0" * 64, "localhost:5000/x", "üñi:latest"]
CAPS = ["NET_ADMIN", "CHOWN", "KILL", "ALL", "SYS_TIME"]


def _maybe(rng, v, p=0.85):
    """v, or a wrongly typed / missing stand-in"""
    r = rng.random()
    if r < p:
        return v
    return rng.choice([None, 7, True, [], {}, "str", 1.5, "__missing__"])


def _container(rng, i):
    c = {}
    name = _maybe(rng, rng.choice(NAMES) + str(i))
    if name != "__missing__":
        c["name"] = name
    img = _maybe(rng, rng.choice(IMAGES))
    if img != "__missing__":
        c["image"] = img
    if rng.random() < 0.7:
        sc = {}
        if rng.random() < 0.5:
            sc["privileged"] = rng.choice([True, False, "true", 1, None])
        if rng.random() < 0.7:
            caps = {}
            for k in ("add", "drop"):
                if rng.random() < 0.6:
                    caps[k] = _maybe(rng, [rng.choice(CAPS + [5, None]) for _ in range(rng.randint(0, 3))])
            sc["capabilities"] = _maybe(rng, caps)
        c["securityContext"] = _maybe(rng, sc)
    return _maybe(rng, c, 0.95)


def _podspec(rng, names):
    spec = {}
    for lst in ("containers", "initContainers", "ephemeralContainers"):
        if rng.random() < (0.9 if lst == "containers" else 0.3):
            spec[lst] = _maybe(rng, [_container(rng, i) for i in range(rng.randint(0, 4))])
    spec["restartPolicy"] = "Always"
    for lst in spec.values():
        if isinstance(lst, list):
            names += [c.get("name") for c in lst if isinstance(c, dict) and isinstance(c.get("name"), str)]
    return _maybe(rng, spec, 0.92)


def _meta(rng, names, labels=True):
    m = {"name": "obj"}
    if labels and rng.random() < 0.8:
        m["labels"] = _maybe(rng, {rng.choice(["app", "env", "tier", "kéy", "a\"q"]) + str(j):
                                   rng.choice(["v1", "prod", 3, None, "été", ""]) for j in range(rng.randint(0, 5))})
    if rng.random() < 0.6:
        ann = {"kubectl.kubernetes.io/last-applied-configuration": "{}"}
        for n in names:
            if rng.random() < 0.6:
                ann["container.apparmor.security.beta.kubernetes.io/" + n] = rng.choice(
                    ["runtime/default", "localhost/p1", "unconfined", 4])
        m["annotations"] = _maybe(rng, ann)
    return _maybe(rng, m, 0.93)


def _doc(rng, raw):
    kind = rng.choice(KINDS)
    names = []
    obj = {"apiVersion": "v1"}
    if kind is not None:
        obj["kind"] = kind
    if kind == "Pod" or (kind is None and rng.random() < 0.5):
        spec = _podspec(rng, names)
        obj["metadata"] = _meta(rng, names)
        obj["spec"] = spec
    elif kind in ("Deployment", "ReplicaSet", "StatefulSet", "DaemonSet", "Job", "ReplicationController"):
        spec = _podspec(rng, names)
        obj["metadata"] = _meta(rng, [], labels=True)
        obj["spec"] = {"replicas": 2, "template": _maybe(rng, {"metadata": _meta(rng, names), "spec": spec}, 0.93)}
    elif kind == "CronJob":
        spec = _podspec(rng, names)
        obj["metadata"] = _meta(rng, [])
        obj["spec"] = {"schedule": "* * * * *", "jobTemplate": {"spec": {"template": {"metadata": _meta(rng, names),
                                                                                   "spec": spec}}}}
    else:
        obj["metadata"] = _meta(rng, [])
    rk = rng.choice(["Pod", "Deployment", "CronJob", "Namespace"])
    req = {"uid": _maybe(rng, "u-%d" % rng.randint(0, 999), 0.97),
           "kind": _maybe(rng, {"group": "", "version": "v1", "kind": rk}, 0.97),
           "resource": _maybe(rng, {"group": "", "version": "v1", "resource": "pods"}, 0.98),
           "operation": _maybe(rng, rng.choice(["CREATE", "UPDATE"]), 0.98),
           "userInfo": _maybe(rng, {"username": "admin"}, 0.98),
           "object": _maybe(rng, obj, 0.95)}
    if rng.random() < 0.8:
        req["namespace"] = _maybe(rng, rng.choice(["default", "kube-system", "né"]), 0.9)
    req = {k: v for k, v in req.items() if v != "__missing__"}
    text = json.dumps({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": req},
                      ensure_ascii=rng.random() < 0.5)
    if rng.random() < 0.05 and '"operation": "' in text:  # a repeated AdmissionRequest field: 422 in both
        text = text.replace('"operation": "', '"operation": "DELETE", "operation": "', 1)
    if rng.random() < 0.1 and '"labels": {' in text:  # a repeated key inside object: the last one counts
        text = text.replace('"labels": {', '"labels": {"app": "dup", ', 1)
    return text


def _product_rows(docs, raw):
    b = K.Batch.from_json(docs, raw=raw)
    v = b.view()
    n = v.n_requests
    arr = lambda p, k: np.ctypeslib.as_array(p, shape=(k,)).copy() if k else np.zeros(0, dtype=np.uint32)
    coff, loff = arr(v.ctr_off, n + 1), arr(v.lbl_off, n + 1)
    nc = int(coff[-1])
    cfl = arr(v.ctr_flags, nc)
    ka, kd = arr(v.capadd_off, nc + 1), arr(v.capdrop_off, nc + 1)

    def col(c, i):
        o = np.ctypeslib.as_array(c.off, shape=(c.n + 1,))
        return bytes(np.ctypeslib.as_array(c.bytes, shape=(int(o[-1]),))[o[i]:o[i + 1]]) if o[-1] else b""
    rows = []
    for r in range(n):
        row = {"flags": int(v.req_flags[r]), "uid": col(v.uid, r), "ns": col(v.ns, r), "op": col(v.op, r),
               "kind": col(v.kind, r), "containers": [], "labels": []}
        for c in range(int(coff[r]), int(coff[r + 1])):
            row["containers"].append((int(cfl[c]), col(v.ctr_name, c), col(v.ctr_image, c), col(v.ctr_apparmor, c),
                                      [col(v.cap_add, k) for k in range(int(ka[c]), int(ka[c + 1]))],
                                      [col(v.cap_drop, k) for k in range(int(kd[c]), int(kd[c + 1]))]))
        for l in range(int(loff[r]), int(loff[r + 1])):
            row["labels"].append((col(v.lbl_key, l), col(v.lbl_val, l)))
        rows.append(row)
    return rows


def _enc(row):
    e = lambda s: s.encode()
    return {"flags": row["flags"], "uid": e(row["uid"]), "ns": e(row["ns"]), "op": e(row["op"]), "kind": e(row["kind"]),
            "containers": [(f, e(n), e(i), e(a), [e(x) for x in ad], [e(x) for x in dr])
                           for f, n, i, a, ad, dr in row["containers"]],
            "labels": [(e(k), e(v)) for k, v in row["labels"]]}


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("raw", [False, True])
def test_flattener_matches_oracle_restatement(seed, raw):
    rng = random.Random(seed * 2 + raw)
    docs = [_doc(rng, raw) for _ in range(300)]
    want = [O.flatten_doc(d, raw=raw) for d in docs]
    ok = [d for d, w in zip(docs, want) if w is not None]
    assert len(ok) > 150
    got = _product_rows(ok, raw)
    for d, g, w in zip(ok, got, [w for w in want if w is not None]):
        assert g == _enc(w), d
    for d, w in zip(docs, want):
        if w is None:  # the oracle rejects the body: so does the product
            with pytest.raises(K.PayloadError):
                K.Batch.from_json([d], raw=raw)
