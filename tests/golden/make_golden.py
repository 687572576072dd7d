"""Write tests/golden/reference_cases.json: the input/expected tables of the reference's own tests
for the hot path, transcribed case by case (each entry cites the reference file:line it comes
from). The reference (Rust) cannot be built or run in this container, so these
literal tables are the pinned golden vectors. Re-run: python tests/golden/make_golden.py

The data files the reference's tests load (tests/data/pod_*.json, raw_review.json) are copied
verbatim into tests/golden/reference_data/.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
MUT = ("Request rejected by policy policy-id. The policy attempted to mutate the request, but it is "
       "currently configured to not allow mutations.")
PATCHED = {"allowed": True, "patch": "patch", "patchType": "JSONPatch"}
REJ500 = {"allowed": False, "status": {"message": "some rejection message", "code": 500}}

cases = {
    # src/evaluation/policy_id.rs:55-73
    "policy_id": [
        {"input": "policy1", "expected": {"policy": "policy1"}, "ref": "policy_id.rs:56"},
        {"input": "group1/policy1", "expected": {"group": "group1", "name": "policy1"}, "ref": "policy_id.rs:57-63"},
        {"input": "", "error": "Not a valid Policy ID: ", "ref": "policy_id.rs:64"},
        {"input": "a/b/c", "error": "Not a valid Policy ID: a/b/c", "ref": "policy_id.rs:65"},
    ],
    # validation_response_with_constraints, policy id "policy-id" (service.rs:221)
    "constraints": [
        {"ref": "service.rs:302-315", "mode": "protect", "a2m": False, "in": PATCHED,
         "out": {"allowed": False, "status": {"message": MUT}}},
        {"ref": "service.rs:317-330", "mode": "monitor", "a2m": False, "in": PATCHED, "out": {"allowed": True}},
        {"ref": "service.rs:340-354", "mode": "monitor", "a2m": True, "in": PATCHED, "out": {"allowed": True}},
        {"ref": "service.rs:356-369", "mode": "monitor", "a2m": False, "in": PATCHED, "out": {"allowed": True}},
        {"ref": "service.rs:371-383", "mode": "monitor", "a2m": True, "in": {"allowed": True}, "out": {"allowed": True}},
        {"ref": "service.rs:385-401", "mode": "monitor", "a2m": True, "in": REJ500, "out": {"allowed": True}},
        {"ref": "service.rs:403-414", "mode": "monitor", "a2m": False, "in": {"allowed": True}, "out": {"allowed": True}},
        {"ref": "service.rs:416-432", "mode": "monitor", "a2m": False, "in": REJ500, "out": {"allowed": True}},
        {"ref": "service.rs:442-461", "mode": "protect", "a2m": True, "in": PATCHED, "out": PATCHED},
        {"ref": "service.rs:463-486", "mode": "protect", "a2m": False, "in": PATCHED,
         "out": {"allowed": False, "status": {"message": MUT}}},
        {"ref": "service.rs:488-500", "mode": "protect", "a2m": True, "in": {"allowed": True}, "out": {"allowed": True}},
        {"ref": "service.rs:502-526", "mode": "protect", "a2m": True, "in": REJ500, "out": REJ500},
        {"ref": "service.rs:528-539", "mode": "protect", "a2m": False, "in": {"allowed": True}, "out": {"allowed": True}},
        {"ref": "service.rs:541-565", "mode": "protect", "a2m": False, "in": REJ500, "out": REJ500},
    ],
    # service::evaluate with a mocked environment (service.rs:568-718); request:
    # test_utils.rs:3-37 (uid "hello", Scale UPDATE in my-namespace). Mock: accepts, or rejects
    # with ("boom", 500); allowed_to_mutate false; always-accept namespace per case.
    "evaluate": [
        {"ref": "service.rs:570", "env": "accept", "mode": "protect", "origin": "validate", "allowed": True},
        {"ref": "service.rs:571", "env": "accept", "mode": "monitor", "origin": "validate", "allowed": True},
        {"ref": "service.rs:572", "env": "accept", "mode": "protect", "origin": "audit", "allowed": True},
        {"ref": "service.rs:573", "env": "accept", "mode": "monitor", "origin": "audit", "allowed": True},
        {"ref": "service.rs:596", "env": "reject", "mode": "protect", "origin": "validate", "allowed": False,
         "status": {"message": "boom", "code": 500}},
        {"ref": "service.rs:597", "env": "reject", "mode": "monitor", "origin": "validate", "allowed": True,
         "status": None},
        {"ref": "service.rs:598", "env": "reject", "mode": "protect", "origin": "audit", "allowed": False,
         "status": {"message": "boom", "code": 500}},
        {"ref": "service.rs:599", "env": "reject", "mode": "monitor", "origin": "audit", "allowed": False,
         "status": {"message": "boom", "code": 500}},
        {"ref": "service.rs:637-654", "env": "accept", "mode": "protect", "origin": "validate", "raw": True,
         "allowed": True},
        {"ref": "service.rs:656-683", "env": "reject", "mode": "protect", "origin": "validate", "raw": True,
         "allowed": False, "status": {"message": "boom", "code": 500}},
        {"ref": "service.rs:687", "env": "reject", "mode": "protect", "origin": "validate",
         "namespace": "kubewarden_special", "always_accept": "kubewarden_special", "allowed": True, "status": None},
        {"ref": "service.rs:688", "env": "reject", "mode": "protect", "origin": "audit",
         "namespace": "kubewarden_special", "always_accept": "kubewarden_special", "allowed": True, "status": None},
    ],
    "admission_review_request": {
        "ref": "test_utils.rs:3-37",
        "request": {
            "uid": "hello", "kind": {"group": "autoscaling", "version": "v1", "kind": "Scale"},
            "resource": {"group": "apps", "version": "v1", "resource": "deployments"}, "subResource": "scale",
            "requestKind": {"group": "autoscaling", "version": "v1", "kind": "Scale"},
            "requestResource": {"group": "apps", "version": "v1", "resource": "deployments"},
            "requestSubResource": "scale", "name": "my-deployment", "namespace": "my-namespace",
            "operation": "UPDATE",
            "userInfo": {"username": "admin", "uid": "014fbff9a07c",
                         "groups": ["system:authenticated", "my-admin-group"],
                         "extra": {"some-key": ["some-value1", "some-value2"]}},
            "object": {"apiVersion": "autoscaling/v1", "kind": "Scale"},
            "oldObject": {"apiVersion": "autoscaling/v1", "kind": "Scale"},
            "options": {"apiVersion": "meta.k8s.io/v1", "kind": "UpdateOptions"}, "dryRun": False}},
    # groups of gatekeeper happy/unhappy members (evaluation_environment.rs:725-937, 979-1042);
    # happy -> [{"result":[]}], unhappy -> [{"result":[{"msg":"failing as expected"}]}]
    "groups": [
        {"ref": "evaluation_environment.rs:980-995", "members": {"happy_policy_1": "happy", "unhappy_policy_1": "unhappy",
                                                                 "unhappy_policy_2": "unhappy"},
         "expression": "unhappy_policy_1() || (happy_policy_1() && unhappy_policy_2())", "allowed": False,
         "causes": [{"field": "spec.policies.unhappy_policy_1", "message": "failing as expected"},
                    {"field": "spec.policies.unhappy_policy_2", "message": "failing as expected"}]},
        {"ref": "evaluation_environment.rs:996-1000", "members": {"happy_policy_1": "happy",
                                                                  "unhappy_policy_1": "unhappy",
                                                                  "unhappy_policy_2": "unhappy"},
         "expression": "unhappy_policy_1() || happy_policy_1() || unhappy_policy_2()", "allowed": True,
         "causes": []},
    ],
    # validate_settings of groups (evaluation_environment.rs:1075-1112, incl. the commented-out
    # "1 + 1" case whose comment says it passes validation)
    "group_expressions": [
        {"ref": "evaluation_environment.rs:788", "members": ["happy_policy_1"], "expression": "true || happy_policy_1()", "valid": True},
        {"ref": "evaluation_environment.rs:796", "members": [], "expression": "2 > 1", "valid": True},
        {"ref": "evaluation_environment.rs:815", "members": ["happy_policy_1"], "expression": "unknown_policy() || happy_policy_1()", "valid": False},
        {"ref": "evaluation_environment.rs:823", "members": [], "expression": "something that doesn't make sense", "valid": False},
        {"ref": "evaluation_environment.rs:832,1093-1097", "members": [], "expression": "1 + 1", "valid": True},
        {"ref": "evaluation_environment.rs:852", "members": ["happy_policy_1"], "expression": "happy_policy_1() + 1", "valid": False},
    ],
    # lookups (evaluation_environment.rs:939-977)
    "lookup": [
        {"ref": "evaluation_environment.rs:940", "policy": "policy_not_defined", "error": "PolicyNotFound"},
        {"ref": "evaluation_environment.rs:941", "policy": "happy_policy_1", "error": None},
    ],
    # policies.yml schema (config.rs:507-730)
    "config": {
        "read_policies_file": {
            "ref": "config.rs:507-588",
            "yaml": "---\nexample:\n    module: ghcr.io/kubewarden/policies/context-aware-policy:0.1.0\n    settings: {}\n"
                    "    allowedToMutate: true\n    contextAwareResources:\n        - apiVersion: v1\n          kind: Namespace\n"
                    "        - apiVersion: v1\n          kind: Pod\ngroup_policy:\n    policyMode: monitor\n"
                    "    expression: \"true\"\n    message: \"group policy message\"\n    policies:\n        policy1:\n"
                    "            module: ghcr.io/kubewarden/policies/policy1:0.1.0\n            settings: {}\n"
                    "        policy2:\n            module: ghcr.io/kubewarden/policies/policy2:0.1.0\n            settings: {}\n",
            "expected": {
                "example": {"kind": "policy", "module": "ghcr.io/kubewarden/policies/context-aware-policy:0.1.0",
                            "policyMode": "protect", "allowedToMutate": True, "settings": {}},
                "group_policy": {"kind": "group", "policyMode": "monitor", "expression": "true",
                                 "message": "group policy message", "members": ["policy1", "policy2"]}}},
        "settings_conversion": [
            {"ref": "config.rs:591-598", "yaml": "---\nexample:\n  module: file:///tmp/namespace-validate-policy.wasm\n  settings: {}\n", "expected": {}},
            {"ref": "config.rs:599-605", "yaml": "---\nexample:\n  module: file:///tmp/namespace-validate-policy.wasm\n", "expected": {}},
            {"ref": "config.rs:606-613", "yaml": "---\nexample:\n  module: file:///tmp/namespace-validate-policy.wasm\n  settings: null\n", "expected": {}},
            {"ref": "config.rs:614-624", "yaml": "---\nexample:\n  module: file:///tmp/namespace-validate-policy.wasm\n  settings:\n    \"counter\": 1\n    \"items\": [\"a\", \"b\"]\n    \"nested\": {\"key\": \"value\"}\n",
             "expected": {"counter": 1, "items": ["a", "b"], "nested": {"key": "value"}}},
        ],
        "policy_validation": [
            {"ref": "config.rs:677-695", "valid": True,
             "yaml": "---\nexample:\n  module: file:///tmp/namespace-validate-policy.wasm\n  settings: {}\ngroup_policy:\n  expression: \"true\"\n  message: \"group policy message\"\n  policies:\n    policy1:\n      module: file:///tmp/namespace-validate-policy.wasm\n      settings: {}\n    policy2:\n      module: file:///tmp/namespace-validate-policy.wasm\n      settings: {}\n"},
            {"ref": "config.rs:696-704", "valid": False,
             "yaml": "---\nexample/invalid:\n  module: file:///tmp/namespace-validate-policy.wasm\n  settings: {}\n"},
            {"ref": "config.rs:705-723", "valid": False,
             "yaml": "---\nexample:\n  module: file:///tmp/namespace-validate-policy.wasm\n  settings: {}\ngroup_policy:\n  expression: \"true\"\n  message: \"group policy message\"\n  policies:\n    policy1/a:\n      module: file:///tmp/namespace-validate-policy.wasm\n      settings: {}\n    policy2:\n      module: file:///tmp/namespace-validate-policy.wasm\n      settings: {}\n"},
        ],
    },
    # HTTP-level strings (tests/integration_test.rs)
    "integration": {
        "privileged_message": {"ref": "integration_test.rs:58-68", "message": "Privileged container is not allowed",
                               "code": None, "fixture": "pod_with_privileged_containers.json"},
        "group_message": {"ref": "integration_test.rs:101-131", "message": "The group policy rejected your request",
                          "causes": 1},
        "group_mutation_cause": {"ref": "integration_test.rs:247-250",
                                 "message": "mutation is not allowed inside of policy group"},
        "not_found_status": {"ref": "integration_test.rs:152", "status": 404},
        "invalid_payload_status": {"ref": "integration_test.rs:171", "status": 422},
        "mutation_refused": {"ref": "service.rs:172", "template": "Request rejected by policy {policy_id}. The policy "
                             "attempted to mutate the request, but it is currently configured to not allow mutations."},
    },
    # error Display strings (errors.rs:5-24) and HTTP mapping (handlers.rs:321-342)
    "errors": {
        "InvalidPolicyId": "Not a valid Policy ID: {0}", "PolicyInitialization": "{0}",
        "PolicyNotFound": "unknown policy: {0}", "BootstrapFailure": "bootstrap failure: {0}",
        "http": {"PolicyNotFound": 404, "other": 500, "other_message": "Something went wrong"},
    },
}


def main():
    with open(os.path.join(HERE, "reference_cases.json"), "w") as f:
        json.dump(cases, f, indent=1, sort_keys=False)
        f.write("\n")


if __name__ == "__main__":
    main()
