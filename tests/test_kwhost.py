"""CPU: the kwhost HTTP front's routing, extractor rejections and error mapping (no device tables:
--no-device, every evaluation answers 500). Reference behaviour: src/lib.rs:206-225 (routes),
handlers.rs:29-39 + api_error.rs (JsonExtractor rejection JSON on /validate, axum's plain-text
rejection on /audit and /validate_raw), handlers.rs:321-342 (404 unknown policy, 500 otherwise),
tests/integration_test.rs:135-370 (404 / 422 cases)."""
import json

import pytest

from helpers import reference_doc
from kwhost_util import Host

POD = reference_doc("pod_with_privileged_containers.json")


@pytest.fixture(scope="module")
def host():
    with Host("parity", extra=["--no-device"]) as h:
        yield h


def test_readiness_and_unknown_routes(host):
    assert host.request("GET", "/readiness")[0] == 200
    assert host.request("GET", "/nope")[0] == 404
    assert host.request("POST", "/validate/")[0] == 404
    assert host.request("GET", "/validate/pod-privileged")[0] == 405
    st, ct, body = host.request("GET", "/metrics")  # no device: nothing evaluated, nothing recorded
    assert st == 200 and ct.startswith("text/plain")
    assert body.decode().splitlines() == ["# TYPE kubewarden_policy_evaluations_total counter",
                                          "# TYPE kubewarden_policy_evaluation_latency_milliseconds histogram"]


@pytest.mark.parametrize("route", ["validate", "audit", "validate_raw"])
def test_unknown_policy_404(host, route):
    st, ct, body = host.request("POST", f"/{route}/does_not_exist", POD)
    assert st == 404 and ct == "application/json"
    assert json.loads(body) == {"message": "unknown policy: does_not_exist", "status": 404}


def test_invalid_policy_id_500(host):
    st, _, body = host.request("POST", "/validate/a%2Fb%2Fc", POD)
    assert st == 500 and json.loads(body) == {"message": "Something went wrong", "status": 500}


def test_validate_invalid_payload_422_json(host):
    st, ct, body = host.request("POST", "/validate/pod-privileged", "{}")
    assert st == 422 and ct == "application/json"
    msg = json.loads(body)
    assert msg["status"] == 422
    assert msg["message"].startswith("Failed to deserialize the JSON body into the target type")


@pytest.mark.parametrize("route", ["audit", "validate_raw"])
def test_plain_extractor_422_text(host, route):
    st, ct, body = host.request("POST", f"/{route}/pod-privileged", "{}")
    assert st == 422 and ct.startswith("text/plain")
    assert body.decode().startswith("Failed to deserialize the JSON body into the target type")


def test_syntax_400_and_media_type_415(host):
    st, _, body = host.request("POST", "/validate/pod-privileged", "{not json")
    assert st == 400 and json.loads(body)["message"].startswith("Failed to parse the request body as JSON")
    st, _, body = host.request("POST", "/validate/pod-privileged", POD, ctype="text/plain")
    assert st == 415
    assert json.loads(body)["message"] == "Expected request with `Content-Type: application/json`"


def test_payload_error_wins_over_unknown_policy(host):
    # the extractor runs before the handler looks the policy up
    assert host.request("POST", "/validate/does_not_exist", "{}")[0] == 422


def test_no_device_answers_500_and_keeps_the_connection(host):
    c = host.conn()
    for _ in range(3):
        st, _, body = host.request("POST", "/validate/pod-privileged", POD, conn=c)
        assert st == 500 and json.loads(body)["status"] == 500
    c.close()


def test_concurrent_mixed_routes(host):
    """Many connections at once across the three routes (the batcher partitions each take by route)."""
    from concurrent.futures import ThreadPoolExecutor
    ids = ["pod-privileged", "namespace_simple", "does_not_exist"]
    routes = ["validate", "audit", "validate_raw"]

    def one(i):
        return host.request("POST", f"/{routes[i % 3]}/{ids[(i // 3) % 3]}", POD)[0]
    with ThreadPoolExecutor(24) as ex:
        res = list(ex.map(one, range(900)))
    assert res.count(404) == 300 and res.count(500) == 600
    assert host.proc.poll() is None


@pytest.mark.parametrize("chunked", [False, True])
@pytest.mark.parametrize("route,json_body", [("validate", True), ("audit", False)])
def test_body_limit_413(host, chunked, route, json_body):
    """axum's DefaultBodyLimit (2 MiB): a larger body is refused with 413 before it is read, on both
    the Content-Length and the chunked path, and the connection closes."""
    big = '{"request": {"uid": "' + "x" * (2 << 20) + '"}}'
    st, ct, body = host.request("POST", f"/{route}/pod-privileged", big, chunked=chunked)
    assert st == 413
    msg = "Failed to buffer the request body: length limit exceeded"
    if json_body:
        assert json.loads(body) == {"message": msg, "status": 413}
    else:
        assert body.decode() == msg and ct.startswith("text/plain")
    assert host.request("GET", "/readiness")[0] == 200  # the server is still serving


def test_reference_policies_yml_example():
    """The reference's own policies.yml.example, verbatim, read by kwhost's native YAML reader
    (config.rs:449-453) under --continue-on-errors: every policy and the group are registered (here
    without device tables their evaluations answer 500; test_kwhost_gpu checks the answers)."""
    from helpers import GOLDEN
    import os
    path = os.path.join(GOLDEN, "reference_data", "policies.yml.example")
    with Host(None, extra=["--no-device"], policies_file=path) as h:
        for pid in ("psp-apparmor", "psp-capabilities"):
            st, _, body = h.request("POST", f"/validate/{pid}", POD)
            assert st == 500, (pid, st, body)
        for pid in ("pod-image-signatures", "pod-image-signatures%2Freject_latest_tag"):
            assert h.request("POST", f"/validate/{pid}", POD)[0] == 500, pid
        assert h.request("POST", "/validate/nope", POD)[0] == 404
