"""CPU: psp-capabilities mutation responses. An accepted
mutation (verdict bit F_PATCH: validate with allowedToMutate, or audit) answers
{uid, allowed: true, patchType: "JSONPatch", patch: base64(RFC 6902 ops)}; the product's patch
(service.cpp capabilities_patch) equals the oracle's restatement byte for byte, and applying it
to the document leaves nothing to mutate. Verdicts come from the host diagnostic walk (the GPU
path is checked in test_kwhost_gpu.py / test_parity_gpu.py). Parity unpinned: the guest's
mutated_object and policy-evaluator's diff are upstream and absent."""
import base64
import copy
import json

import numpy as np
import pytest

import kwgpu as K
import oracle as O

CAPS = "registry://ghcr.io/kubewarden/policies/psp-capabilities:v0.1.7"
POLICIES = {
    "caps-mutate": {"module": CAPS, "allowedToMutate": True,
                    "settings": {"allowed_capabilities": ["*"], "required_drop_capabilities": ["KILL", "NET_RAW"],
                                 "default_add_capabilities": ["CHOWN", "SETUID"]}},
    "caps-drop-only": {"module": CAPS, "allowedToMutate": True,
                       "settings": {"allowed_capabilities": ["NET_ADMIN", "CHOWN"],
                                    "required_drop_capabilities": ["KILL", "KILL"]}},
    "caps-refused": {"module": CAPS, "settings": {"allowed_capabilities": ["*"],
                                                  "default_add_capabilities": ["AUDIT_WRITE"]}},
}

CONTAINERS = [
    {"name": "bare", "image": "nginx"},
    {"name": "sc-no-caps", "image": "nginx", "securityContext": {"privileged": False}},
    {"name": "caps-empty", "image": "nginx", "securityContext": {"capabilities": {}}},
    {"name": "drop-kill", "image": "nginx", "securityContext": {"capabilities": {"drop": ["KILL"]}}},
    {"name": "drop-all", "image": "nginx", "securityContext": {"capabilities": {"drop": ["ALL"], "add": ["CHOWN"]}}},
    {"name": "full", "image": "nginx",
     "securityContext": {"capabilities": {"drop": ["KILL", "NET_RAW"], "add": ["CHOWN", "SETUID"]}}},
    {"name": "add-null", "image": "nginx", "securityContext": {"capabilities": {"add": None, "drop": ["NET_RAW"]}}},
    "not-an-object",
]


def review(uid, obj, kind="Pod"):
    return json.dumps({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                       "request": {"uid": uid, "kind": {"group": "", "version": "v1", "kind": kind},
                                   "resource": {"group": "", "version": "v1", "resource": "pods"},
                                   "operation": "CREATE", "userInfo": {}, "namespace": "default", "object": obj}})


def documents():
    docs = []
    for i, c in enumerate(CONTAINERS):
        docs.append(review(f"p{i}", {"kind": "Pod", "metadata": {"name": "x"}, "spec": {"containers": [c]}}))
    spec = {"containers": CONTAINERS[:3], "initContainers": [CONTAINERS[3], CONTAINERS[7], CONTAINERS[0]],
            "ephemeralContainers": [CONTAINERS[5], CONTAINERS[1]]}
    docs.append(review("multi", {"kind": "Pod", "spec": copy.deepcopy(spec)}))
    docs.append(review("deploy", {"kind": "Deployment", "spec": {"template": {"spec": copy.deepcopy(spec)}}},
                       kind="Deployment"))
    docs.append(review("cron", {"kind": "CronJob", "spec": {"jobTemplate": {"spec": {"template": {
        "spec": copy.deepcopy(spec)}}}}}, kind="CronJob"))
    docs.append(review("nothing", {"kind": "Pod", "spec": {"containers": [CONTAINERS[5]]}}))
    return docs


def apply_patch(doc, ops):
    """Minimal RFC 6902 'add' (object member or array append) on request.object."""
    root = json.loads(doc)
    obj = root["request"]["object"]
    for op in ops:
        assert op["op"] == "add"
        parts = op["path"].split("/")[1:]
        tgt = obj
        for p in parts[:-1]:
            tgt = tgt[int(p)] if isinstance(tgt, list) else tgt[p]
        last = parts[-1]
        if last == "-":
            tgt.append(op["value"])
        else:
            tgt[last] = op["value"]
    return json.dumps(root)


@pytest.mark.parametrize("origin", [K.VALIDATE, K.AUDIT])
def test_patch_matches_oracle_and_applies(origin):
    env = K.EvaluationEnvironment(POLICIES)
    oe = O.OracleEnv(POLICIES)
    ids = env.policy_ids()
    docs = documents()
    b = K.Batch.from_json(docs)
    v = b.debug_host_walk(env, ids, origin).reshape(len(docs), len(ids))
    assert np.array_equal(v.ravel(), oe.eval(b.view(), ids, origin))
    patched = 0
    for r, doc in enumerate(docs):
        for j, pid in enumerate(ids):
            w = int(v[r, j])
            got = b.format_response(env, r, j, w, doc=doc)
            want = oe.response_doc(b.view(), r, j, origin, doc=doc)
            assert got == want, (pid, r, got, want)
            if not w & K._native.KW_F_PATCH:
                continue
            patched += 1
            ops = json.loads(base64.b64decode(got["patch"]))
            assert ops, (pid, r)
            fixed = apply_patch(doc, ops)
            fb = K.Batch.from_json([fixed])
            fv = int(fb.debug_host_walk(env, [pid], origin)[0])
            assert not fv & K._native.KW_V_MUTATED, (pid, r, ops)
    assert patched >= 10


def test_patch_requires_the_document():
    env = K.EvaluationEnvironment(POLICIES)
    ids = env.policy_ids()
    b = K.Batch.from_json(documents()[:1])
    w = int(b.debug_host_walk(env, ids[:1], K.AUDIT)[0])
    assert w & K._native.KW_F_PATCH
    with pytest.raises(K.EvaluationError):
        b.format_response(env, 0, 0, w)


def test_refused_mutation_has_no_patch():
    env = K.EvaluationEnvironment(POLICIES)
    ids = env.policy_ids()
    j = ids.index("caps-refused")
    docs = documents()
    b = K.Batch.from_json(docs)
    w = int(b.debug_host_walk(env, [ids[j]], K.VALIDATE)[0])
    got = b.format_response(env, 0, j, w, doc=docs[0])
    assert got["allowed"] is False and "patch" not in got
    assert got["status"]["message"].startswith("Request rejected by policy caps-refused.")
