"""GPU: the kwhost HTTP front end to end. Concurrent /validate, /audit and /validate_raw calls
(the micro-batcher groups them into kw_validate_rows passes) answer exactly the oracle's
AdmissionResponse inside the reference envelope (AdmissionReviewResponse, admission_review.rs:28-35;
RawReviewResponse, raw_review.rs), or the reference's 404 where the service layer raises
PolicyNotFound (handlers.rs:321-342)."""
import json
from concurrent.futures import ThreadPoolExecutor
from urllib.parse import quote

import pytest

import kwgpu as K
import oracle as O
from helpers import config, reference_doc
from kwhost_util import Host

pytestmark = pytest.mark.gpu
NS = "kubewarden"


def _expect(oe, soa, origin, r, j, raw, doc):
    try:
        resp = oe.response_doc(soa, r, j, origin, doc=doc)
    except KeyError as e:
        return 404, {"message": str(e).strip("'\""), "status": 404}
    if raw:
        return 200, {"response": resp}
    return 200, {"kind": "AdmissionReview", "apiVersion": "admission.k8s.io/v1", "response": resp}


@pytest.mark.parametrize("name,scfg,pipes", [("parity", 0, 1), ("c4_64", 4, 1), ("c4_64", 4, 2)],
                         ids=["parity", "c4_64", "c4_64-two-pipelines"])
def test_concurrent_routes_match_oracle(name, scfg, pipes):
    """pipes = 2 (r06): `--devices 0,0` — the serving front sharded over two device
    pipelines, the second environment deserialized from the first one's blob (kw_env_serialize /
    kw_env_deserialize, as for the RCCL broadcast), both serving batches."""
    doc = config(name)
    oe = O.OracleEnv(doc, continue_on_errors=True, always_accept_namespace=NS)
    ids = [p["id"] for p in oe.pol]
    n = 240
    syn = K.SynthBatch(scfg, n, seed=31337 + scfg)
    docs = [syn.json(r) for r in range(n)]
    soa = syn.soa()
    raw_b = K.Batch.from_json(docs, raw=True)
    raw_soa = raw_b.view()
    calls = []
    for r in range(n):
        j = (r * 7) % len(ids)
        calls.append(("validate", r, j, _expect(oe, soa, K.VALIDATE, r, j, False, docs[r])))
        calls.append(("audit", r, j, _expect(oe, soa, K.AUDIT, r, j, False, docs[r])))
        calls.append(("validate_raw", r, j, _expect(oe, raw_soa, K.VALIDATE, r, j, True, docs[r])))
    dev = ["--device", "0"] if pipes == 1 else ["--devices", ",".join(["0"] * pipes), "--stats-ms", "100"]
    with Host(name, extra=dev + ["--max-wait-us", "300"]) as h:
        def one(c):
            route, r, j, want = c
            # member ids ("group/member") travel percent-encoded, as axum's Path extractor decodes them
            st, _, body = h.request("POST", f"/{route}/{quote(ids[j], safe='')}", docs[r])
            return c, st, json.loads(body) if body else None
        with ThreadPoolExecutor(max_workers=24) as ex:
            results = list(ex.map(one, calls))
        st, _, metrics = h.request("GET", "/metrics")
        if pipes > 1:
            import time
            time.sleep(0.3)  # one more stats line after the last batch
            stats = [json.loads(line)["kwhost_stats"] for line in h.stderr().splitlines() if "kwhost_stats" in line]
            per_dev = stats[-1]["device_batches"]
            assert len(per_dev) == pipes and all(b > 0 for b in per_dev), per_dev
    assert st == 200
    # every evaluated call (200) is one kubewarden_policy_evaluations_total data point (service.rs:40-150)
    total = sum(int(line.rsplit(" ", 1)[1]) for line in metrics.decode().splitlines()
                if line.startswith("kubewarden_policy_evaluations_total{"))
    assert total == sum(1 for _, st, _ in results if st == 200)
    bad = [(c[0], c[1], ids[c[2]], st, got, c[3]) for c, st, got in results if (st, got) != c[3]]
    assert not bad, bad[:3]
    assert sum(1 for c in calls if c[3][0] == 200) > len(calls) // 2
    if name == "parity":  # accepted mutations (audit / allowedToMutate) came back with their patch
        assert any(c[3][0] == 200 and "patch" in c[3][1].get("response", {}) for c in calls)


def test_reference_fixture_privileged_pod():
    """integration_test.rs:58-68: pod-privileged rejects tests/data/pod_with_privileged_containers.json
    with "Privileged container is not allowed" and no code; the unprivileged pod is accepted."""
    with Host("parity", extra=["--device", "0"]) as h:
        st, _, body = h.request("POST", "/validate/pod-privileged", reference_doc("pod_with_privileged_containers.json"))
        assert st == 200
        resp = json.loads(body)["response"]
        assert resp["allowed"] is False
        assert resp["status"] == {"message": "Privileged container is not allowed"}
        st, _, body = h.request("POST", "/validate/pod-privileged",
                                reference_doc("pod_without_privileged_containers.json"))
        assert st == 200 and json.loads(body)["response"]["allowed"] is True


def test_reference_policies_yml_example_served():
    """The reference's policies.yml.example, verbatim, through kwhost's native YAML reader under
    --continue-on-errors: psp-capabilities (allowedToMutate, required drop KILL) answers the oracle's
    response (a JSONPatch adding the drop), psp-apparmor accepts, the trusted-repos member answers
    as a policy, and the group whose verify-image-signatures members are not declarative (their
    initialisation failed) answers 404 for its first broken member (service.rs:73-94)."""
    import os

    import yaml
    from helpers import GOLDEN
    path = os.path.join(GOLDEN, "reference_data", "policies.yml.example")
    with open(path) as f:
        doc = yaml.safe_load(f)
    oe = O.OracleEnv(doc, continue_on_errors=True)
    pod = reference_doc("pod_with_privileged_containers.json")
    b = K.Batch.from_json([pod])
    with Host(None, extra=["--device", "0"], policies_file=path, namespace=None) as h:
        for pid in ("psp-apparmor", "psp-capabilities", "pod-image-signatures/reject_latest_tag"):
            st, _, body = h.request("POST", f"/validate/{quote(pid, safe='')}", pod)
            assert st == 200, (pid, body)
            want = oe.response_doc(b.view(), 0, oe.ids[pid], K.VALIDATE, doc=pod)
            assert json.loads(body)["response"] == want, pid
        st, _, body = h.request("POST", "/validate/pod-image-signatures", pod)
        assert st == 404 and json.loads(body)["message"] == "unknown policy: pod-image-signatures/sigstore_pgp"
    assert "patch" in oe.response_doc(b.view(), 0, oe.ids["psp-capabilities"], K.VALIDATE, doc=pod)
