"""Generate the policies.yml documents of the benchmark / parity configurations.

  c1_namespace.yml   C1 namespace_simple: namespace-validate-policy, valid_namespace kubewarden-approved
  c2_trusted.yml     C2 trusted-repos: registries.allow [ghcr.io, quay.io, registry.k8s.io], tags.reject [latest]
  c3_group.yml       C3 group: two image-glob stand-ins for the sigstore members + reject_latest_tag,
                     expression "sigstore_pgp() || (sigstore_gh_action() && reject_latest_tag())"
                     (policies.yml.example:9-33; verify-image-signatures is not declarative)
  c4_64.yml          C4: 64 policies = 22 psp-capabilities (validate-only settings, a third with
                     required_drop so the mutation-refused path is live) + 21 psp-apparmor + 21 safe-labels
  c5_mixed.yml       C5: the C4 policy set (served on the mixed Pod/Deployment/Namespace stream)
  c6_256.yml         256 policies past every per-column pattern count of a 64-bit design: 64 trusted-repos
                     over 240 registries (literals and globs) and 230 image globs, 64 psp-capabilities,
                     48 psp-apparmor over 101 profiles, 40 safe-labels over 150 label keys, 24
                     namespace-validate, 15 pod-privileged and a 40-member group (synth config 6)
  parity.yml         every family, monitor mode, allowedToMutate, groups (incl. an i64 expression),
                     an unsupported module and invalid settings (load with continue_on_errors)
Deterministic (seeded); run `python configs/gen_configs.py` to regenerate.
"""
import os
import random

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
CAPS = ["NET_ADMIN", "SYS_TIME", "SYS_ADMIN", "NET_RAW", "CHOWN", "KILL", "SETUID", "SETGID", "DAC_OVERRIDE",
        "FOWNER", "MKNOD", "AUDIT_WRITE", "SYS_PTRACE", "NET_BIND_SERVICE"]
PROFILES = ["runtime/default", "unconfined"] + [f"localhost/p{i}" for i in range(10)]
KEYS = ["app", "tier", "env", "team", "owner", "version", "release", "component", "part-of", "managed-by",
        "app.kubernetes.io/name", "app.kubernetes.io/instance", "app.kubernetes.io/version",
        "app.kubernetes.io/component", "app.kubernetes.io/part-of", "app.kubernetes.io/managed-by", "cost-center",
        "region", "zone", "critical", "debug", "experimental", "legacy", "pci"]
REGEXES = ["^[a-z0-9-]+$", "^v[0-9]+(\\.[0-9]+)*", "^(dev|staging|prod)$", "^team-[a-z]+$", "[0-9]{3,}",
           "^(true|false)$", "^[a-z]{1,8}$", "^(eu|us)-(west|east)-[0-9]$", "^(frontend|backend|db|cache|web)$",
           "^[A-Za-z0-9_.-]{1,63}$", "payments|web", "^x$"]
MOD = {
    "caps": "registry://ghcr.io/kubewarden/policies/psp-capabilities:v0.1.7",
    "aa": "registry://ghcr.io/kubewarden/policies/psp-apparmor:v0.1.7",
    "labels": "registry://ghcr.io/kubewarden/policies/safe-labels:v0.1.14",
    "trusted": "registry://ghcr.io/kubewarden/policies/trusted-repos-policy:v0.1.12",
    "ns": "file:///tmp/namespace-validate-policy.wasm",
    "priv": "registry://ghcr.io/kubewarden/tests/pod-privileged:v0.2.1",
}


def c4_policies(rng):
    pols = {}
    for i in range(22):
        s = {"allowed_capabilities": sorted(rng.sample(CAPS, rng.randint(3, 10)))}
        if i % 3 == 0:
            s["required_drop_capabilities"] = ["KILL"]
        pols[f"psp-capabilities-{i:02d}"] = {"module": MOD["caps"], "settings": s}
    for i in range(21):
        pols[f"psp-apparmor-{i:02d}"] = {"module": MOD["aa"],
                                         "settings": {"allowed_profiles": sorted(rng.sample(PROFILES, rng.randint(2, 8)))}}
    for i in range(21):
        keys = rng.sample(KEYS, 5)
        s = {"denied_labels": keys[:rng.randint(1, 2)]}
        mand = keys[2:2 + rng.randint(0, 1)]
        if mand:
            s["mandatory_labels"] = mand
        s["constrained_labels"] = {k: rng.choice(REGEXES) for k in keys[3:3 + rng.randint(1, 2)]}
        pols[f"safe-labels-{i:02d}"] = {"module": MOD["labels"], "settings": s}
    return pols


REG6 = [f"reg-{i:03d}.example.com" for i in range(240)]
IMG6 = [f"reg-{i:03d}.example.com/team-{i % 40:02d}/*" for i in range(230)]
PROF6 = ["runtime/default"] + [f"localhost/prof-{i:02d}" for i in range(100)]
KEYS6 = [f"team.example/k-{i:03d}" for i in range(150)]


def c6_policies(rng):
    pols = {}
    for i in range(64):
        s = {"registries": {"allow": sorted(rng.sample(REG6, rng.randint(8, 24))) + (["*.corp.example", "reg-1?0.example.com"]
                                                                                   if i % 8 == 0 else [])},
             "tags": {"reject": ["latest"] if i % 2 else ["latest", "*-rc*"]}}
        if i % 4 == 0:
            s["images"] = {"allow": sorted(rng.sample(IMG6, 16))}
        elif i % 4 == 1:
            s["images"] = {"reject": sorted(rng.sample(IMG6, 16))}
        pols[f"trusted-repos-{i:02d}"] = {"module": MOD["trusted"], "settings": s}
    for i in range(64):
        s = {"allowed_capabilities": sorted(rng.sample(CAPS, rng.randint(3, 10)))}
        if i % 3 == 0:
            s["required_drop_capabilities"] = ["KILL"]
        pols[f"psp-capabilities-{i:02d}"] = {"module": MOD["caps"], "settings": s}
    for i in range(48):
        pols[f"psp-apparmor-{i:02d}"] = {"module": MOD["aa"],
                                         "settings": {"allowed_profiles": sorted(rng.sample(PROF6, rng.randint(4, 30)))}}
    for i in range(40):
        keys = rng.sample(KEYS6 + KEYS, 8)
        s = {"denied_labels": keys[:rng.randint(1, 3)]}
        mand = keys[3:3 + rng.randint(0, 2)]
        if mand:
            s["mandatory_labels"] = mand
        s["constrained_labels"] = {k: rng.choice(REGEXES) for k in keys[5:5 + rng.randint(1, 3)]}
        pols[f"safe-labels-{i:02d}"] = {"module": MOD["labels"], "settings": s}
    for i in range(24):
        pols[f"namespace-{i:02d}"] = {"module": MOD["ns"], "settings": {"valid_namespace": f"ns-{i:03d}"}}
    for i in range(15):
        pols[f"pod-privileged-{i:02d}"] = {"module": MOD["priv"], "settings": {"skip_init_containers": i % 2 == 1}}
    members = {}
    for m in range(40):
        if m % 2 == 0:
            members[f"m{m:02d}"] = {"module": MOD["trusted"], "settings": {"registries": {"allow": sorted(rng.sample(REG6, 40))}}}
        elif m % 4 == 1:
            members[f"m{m:02d}"] = {"module": MOD["labels"], "settings": {"mandatory_labels": [rng.choice(KEYS)]}}
        else:
            members[f"m{m:02d}"] = {"module": MOD["aa"], "settings": {"allowed_profiles": sorted(rng.sample(PROF6, 20))}}
    clauses = [f"(m{m:02d}() && m{m + 1:02d}())" for m in range(0, 40, 2)]
    pols["group-40"] = {"policies": members, "expression": " || ".join(clauses),
                        "message": "none of the 40-member clauses accepted the request"}
    return pols


def main():
    rng = random.Random(4)
    docs = {
        "c1_namespace.yml": {"namespace_simple": {"module": MOD["ns"], "settings": {"valid_namespace": "kubewarden-approved"}}},
        "c2_trusted.yml": {"trusted-repos": {"module": MOD["trusted"], "settings": {
            "registries": {"allow": ["ghcr.io", "quay.io", "registry.k8s.io"]}, "tags": {"reject": ["latest"]}}}},
        "c3_group.yml": {"pod-image-signatures": {
            "policies": {
                "sigstore_pgp": {"module": MOD["trusted"], "settings": {"images": {"allow": ["ghcr.io/*", "quay.io/*/*:*"]}}},
                "sigstore_gh_action": {"module": MOD["trusted"], "settings": {"registries": {"allow": ["registry.k8s.io", "gcr.io", "quay.io"]}}},
                "reject_latest_tag": {"module": MOD["trusted"], "settings": {"tags": {"reject": ["latest"]}}},
            },
            "expression": "sigstore_pgp() || (sigstore_gh_action() && reject_latest_tag())",
            "message": "The group policy is rejected."}},
        "c4_64.yml": c4_policies(rng),
    }
    docs["c5_mixed.yml"] = docs["c4_64.yml"]
    docs["c6_256.yml"] = c6_policies(random.Random(6))
    prng = random.Random(0)
    parity = {
        "pod-privileged": {"module": MOD["priv"]},
        "pod-privileged-skip-init": {"module": MOD["priv"], "settings": {"skip_init_containers": True,
                                                                         "skip_ephemeral_containers": True}},
        "namespace_simple": {"module": MOD["ns"], "settings": {"valid_namespace": "kubewarden-approved"}},
        "trusted-repos": {"module": MOD["trusted"], "settings": {
            "registries": {"allow": ["ghcr.io", "quay.io", "registry.k8s.io"]}, "tags": {"reject": ["latest"]}}},
        "trusted-images": {"module": MOD["trusted"], "policyMode": "monitor", "settings": {
            "registries": {"reject": ["my-corp.example:*", "gcr.[i]o"]}, "tags": {"reject": ["0.*", "*.1[0-9].*"]},
            "images": {"reject": ["docker.io/library/*", "*/a?c*"]}}},
        "trusted-allow-images": {"module": MOD["trusted"], "settings": {"images": {"allow": [
            "ghcr.io/*", "docker.io/library/*:latest", "*@sha256:*", "quay.io/[!x]*"]}}},
        "psp-capabilities": {"module": MOD["caps"], "allowedToMutate": False, "settings": {
            "allowed_capabilities": ["NET_ADMIN", "CHOWN", "KILL"], "required_drop_capabilities": ["SYS_ADMIN"],
            "default_add_capabilities": ["NET_BIND_SERVICE"]}},
        "psp-capabilities-all": {"module": MOD["caps"], "settings": {"allowed_capabilities": ["*"]}},
        "psp-capabilities-strict": {"module": MOD["caps"], "settings": {"allowed_capabilities": ["CHOWN"]}},
        "psp-apparmor": {"module": MOD["aa"], "settings": {"allowed_profiles": ["runtime/default", "localhost/p1"]}},
        "psp-apparmor-none": {"module": MOD["aa"]},
        "safe-labels": {"module": MOD["labels"], "settings": {
            "denied_labels": ["debug", "legacy"], "mandatory_labels": ["app", "team"],
            "constrained_labels": {"env": "^(dev|staging|prod)$", "version": "^v[0-9]+(\\.[0-9]+)*$"}}},
        "safe-labels-monitor": {"module": MOD["labels"], "policyMode": "monitor", "settings": {
            "mandatory_labels": ["app"], "constrained_labels": {"tier": "^(frontend|backend)$"}}},
        "group-or": {"policies": {
            "priv": {"module": MOD["priv"]},
            "reg": {"module": MOD["trusted"], "settings": {"registries": {"allow": ["ghcr.io"]}}},
            "latest": {"module": MOD["trusted"], "settings": {"tags": {"reject": ["latest"]}}}},
            "expression": "reg() || (priv() && latest())", "message": "The group policy rejected your request"},
        "group-mixed": {"policyMode": "monitor", "policies": {
            "aa": {"module": MOD["aa"], "settings": {"allowed_profiles": ["runtime/default"]}},
            "lbl": {"module": MOD["labels"], "settings": {"mandatory_labels": ["app"]}},
            "caps": {"module": MOD["caps"], "settings": {"allowed_capabilities": ["CHOWN"], "required_drop_capabilities": ["KILL"]}}},
            "expression": "!(aa() == lbl()) || caps() != false && 3 > 2", "message": "mixed group"},
        "group-int": {"policies": {"a": {"module": MOD["priv"]}}, "expression": "1 + 1", "message": "int group"},
        "group-invalid": {"policies": {"a": {"module": MOD["priv"]}}, "expression": "a() + 1", "message": "bad"},
        "unsupported": {"module": "registry://ghcr.io/kubewarden/policies/verify-image-signatures:v0.2.8"},
        "bad-settings": {"module": MOD["trusted"], "settings": {"registries": {"allow": ["a"], "reject": ["b"]}}},
    }
    docs["parity.yml"] = parity
    del prng
    for name, doc in docs.items():
        with open(os.path.join(HERE, name), "w") as f:
            f.write(f"# generated by configs/gen_configs.py — {name}\n")
            yaml.safe_dump(doc, f, sort_keys=False, width=120)


if __name__ == "__main__":
    main()
