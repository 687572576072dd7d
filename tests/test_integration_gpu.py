"""The reference's HTTP-level integration tests (tests/integration_test.rs), replayed through
kw_evaluate (service::evaluate + the GPU hot path) with the same fixtures and expected strings.
Policies outside the declarative class (raw-mutation-policy, sleeping-policy) have no analogue;
their tests are mapped as noted per test.
"""
import pytest

import kwgpu as K
from helpers import reference_doc

pytestmark = pytest.mark.gpu

# default_test_config (tests/common/mod.rs:29-131), restricted to the declarative class
CONFIG = {
    "pod-privileged": {"module": "ghcr.io/kubewarden/tests/pod-privileged:v0.2.1"},
    "group-policy-just-pod-privileged": {
        "expression": "pod_privileged() && true",
        "message": "The group policy rejected your request",
        "policyMode": "protect",
        "policies": {"pod_privileged": {"module": "ghcr.io/kubewarden/tests/pod-privileged:v0.2.1"}},
    },
}


@pytest.fixture(scope="module")
def env():
    return K.EvaluationEnvironment(CONFIG, device=0)


def test_validate(env):
    """integration_test.rs:36-69"""
    resp = env.evaluate("pod-privileged", reference_doc("pod_with_privileged_containers.json"))
    assert resp["allowed"] is False
    assert resp["status"] == {"message": "Privileged container is not allowed"}  # code None
    assert resp["uid"] == "1299d386-525b-4032-98ae-1949f69f9cfc"


@pytest.mark.parametrize("fixture,expected_allowed", [
    ("pod_with_privileged_containers.json", False),
    ("pod_without_privileged_containers.json", True),
])
def test_validate_policy_group(env, fixture, expected_allowed):
    """integration_test.rs:71-132"""
    resp = env.evaluate("group-policy-just-pod-privileged", reference_doc(fixture))
    assert resp["allowed"] is expected_allowed
    assert "warnings" not in resp
    if expected_allowed:
        assert "status" not in resp
    else:
        assert resp["status"]["message"] == "The group policy rejected your request"
        causes = resp["status"]["details"]["causes"]
        assert len(causes) == 1
        assert causes[0]["message"] == "Privileged container is not allowed"
        assert causes[0]["field"] == "spec.policies.pod_privileged"


def test_validate_policy_not_found(env):
    """integration_test.rs:134-153 -> 404"""
    with pytest.raises(K.PolicyNotFound) as e:
        env.evaluate("does_not_exist", reference_doc("pod_with_privileged_containers.json"))
    assert K.http_status(e.value.code) == 404


def test_validate_invalid_payload(env):
    """integration_test.rs:155-172 -> 422"""
    with pytest.raises(K.PayloadError) as e:
        env.evaluate("pod-privileged", "{}")
    assert K.http_status(e.value.code) == 422


def test_audit(env):
    """integration_test.rs:319-344"""
    resp = env.evaluate("pod-privileged", reference_doc("pod_with_privileged_containers.json"), origin=K.AUDIT)
    assert resp["allowed"] is False
    assert resp["status"] == {"message": "Privileged container is not allowed"}


def test_audit_policy_not_found(env):
    with pytest.raises(K.PolicyNotFound):
        env.evaluate("does_not_exist", reference_doc("pod_with_privileged_containers.json"), origin=K.AUDIT)


def test_raw_request(env):
    """integration_test.rs:174-202 uses raw-mutation-policy (not declarative). Here: a raw review
    through a declarative policy is evaluated (no pod spec -> accepted)."""
    resp = env.evaluate("pod-privileged", reference_doc("raw_review.json"), raw=True)
    assert resp == {"uid": "", "allowed": True}


def test_policy_with_invalid_settings():
    """integration_test.rs:482-528: continue_on_errors, invalid settings -> 200 with reject 500
    whose message starts with 'Policy settings are invalid:'."""
    cfg = dict(CONFIG)
    cfg["invalid_settings"] = {"module": "registry://ghcr.io/kubewarden/policies/trusted-repos-policy:v0.1.12",
                               "settings": {"registries": {"allow": "ghcr.io"}}}
    env = K.EvaluationEnvironment(cfg, continue_on_errors=True, device=0)
    resp = env.evaluate("invalid_settings", reference_doc("pod_sleep_100ms.json"))
    assert resp["allowed"] is False
    assert resp["status"]["code"] == 500
    assert resp["status"]["message"].startswith("Policy settings are invalid:")


def test_policy_with_wrong_url():
    """integration_test.rs:530-573: a module the engine cannot serve -> 200, reject 500 on /audit."""
    cfg = dict(CONFIG)
    cfg["wrong_url"] = {"module": "ghcr.io/kubewarden/tests/not_existing:v0.1.0"}
    env = K.EvaluationEnvironment(cfg, continue_on_errors=True, device=0)
    resp = env.evaluate("wrong_url", reference_doc("pod_sleep_100ms.json"), origin=K.AUDIT)
    assert resp["allowed"] is False
    assert resp["status"]["code"] == 500
    assert "wrong_url" in resp["status"]["message"]


def test_namespace_bypass():
    """service.rs:685-718: request from the always-accepted namespace -> allowed, no status."""
    env = K.EvaluationEnvironment(CONFIG, always_accept_namespace="default", device=0)
    for origin in (K.VALIDATE, K.AUDIT):
        resp = env.evaluate("pod-privileged", reference_doc("pod_with_privileged_containers.json"), origin=origin)
        assert resp == {"uid": "1299d386-525b-4032-98ae-1949f69f9cfc", "allowed": True}
