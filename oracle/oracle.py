"""oracle.py — CPU restatement of the hot path, Python half. TEST INFRASTRUCTURE ONLY.

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker or the timed CPU baseline; never by the product (policy-server_amd/kwgpu never imports it).

Restates, independently of the product's C++ (env.cpp / expr.cpp / service.cpp):
  * PolicyID::from_str / Display                     src/evaluation/policy_id.rs:20-47
  * policies document schema + validate_policies      src/config.rs:237-258, 287-453
  * EvaluationEnvironmentBuilder::build (continue_on_errors, member Protect/no-mutate)
                                                      src/evaluation/evaluation_environment.rs:198-365
  * validation_response_with_constraints              src/api/service.rs:160-208
  * service::evaluate response shapes                 src/api/service.rs:30-152
  * PolicyGroupEvaluator expression language (rhai subset, short-circuit) [upstream rhai 1.21.0],
    as pinned by evaluation_environment.rs:979-1112 and integration_test.rs:101-131, 204-251
  * policy-family settings rules and message templates: DESIGN.md §Policy families — parity
    UNPINNED for the families (their Wasm source is not in /root/reference), except the
    pod-privileged message pinned by integration_test.rs:58-68.
  * the psp-capabilities mutation as an RFC 6902 patch — parity UNPINNED (the
    guest's mutated_object and policy-evaluator's diff are upstream, absent here).
The per-request family arithmetic runs in oracle/kworacle.c (the oracle's own glob and regex
matcher, oracle/kwregex.c).
"""
import base64
import ctypes as C
import json
import os
import re

import numpy as np

try:
    from . import rhaisub  # noqa: F401  (package import)
except ImportError:
    import rhaisub

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libkworacle.so")

PROTECT, MONITOR = 0, 1
VALIDATE, AUDIT = 0, 1
F_PRIV, F_NS, F_TRUSTED, F_CAPS, F_AA, F_LABELS, F_GROUP = 1, 2, 3, 4, 5, 6, 7
X_CONST, X_CALL, X_NOT, X_AND, X_OR, X_EQ, X_NE = 0, 1, 2, 3, 4, 5, 6

R_PRIVILEGED, R_NAMESPACE, R_REG_NOT_ALLOWED, R_REG_REJECTED, R_TAG_REJECTED = 1, 2, 3, 4, 5
R_IMG_NOT_ALLOWED, R_IMG_REJECTED, R_CAP, R_APPARMOR = 6, 7, 8, 9
R_LABEL_DENIED, R_LABEL_CONSTRAINT, R_LABEL_MANDATORY, R_GROUP, R_GROUP_EXPR, R_INIT = 10, 11, 12, 13, 14, 15


# ----------------------------------------------------------------------------- mutation patch
_WORKLOADS = ("Deployment", "ReplicaSet", "StatefulSet", "DaemonSet", "Job", "ReplicationController")


def podspec(doc_obj):
    """(PodSpec dict, JSON Pointer) of request.object, or (None, None): Pod /spec, workload templates
    /spec/template/spec, CronJob /spec/jobTemplate/spec/template/spec (object kind, else
    request.kind.kind)."""
    req = doc_obj.get("request") if isinstance(doc_obj, dict) else None
    obj = req.get("object") if isinstance(req, dict) else None
    if not isinstance(obj, dict):
        return None, None
    rk = req.get("kind", {}).get("kind") if isinstance(req.get("kind"), dict) else None
    kind = obj["kind"] if isinstance(obj.get("kind"), str) else (rk if isinstance(rk, str) else "")

    def walk(o, keys):
        for k in keys:
            if not isinstance(o, dict):
                return None
            o = o.get(k)
        return o
    if kind == "Pod":
        spec, ptr = obj.get("spec"), "/spec"
    elif kind in _WORKLOADS:
        spec, ptr = walk(obj, ["spec", "template", "spec"]), "/spec/template/spec"
    elif kind == "CronJob":
        spec, ptr = walk(obj, ["spec", "jobTemplate", "spec", "template", "spec"]), "/spec/jobTemplate/spec/template/spec"
    else:
        return None, None
    return (spec, ptr) if isinstance(spec, dict) else (None, None)


# ----------------------------------------------------------------------------- document -> row
class _Obj(list):
    """A JSON object as its member list in document order (duplicate keys kept, as the product's
    tape keeps them); get() answers the last occurrence, as serde does."""

    def get(self, k, default=None):
        for key, v in reversed(self):
            if key == k:
                return v
        return default


_REQ_FIELDS = ("uid", "kind", "resource", "subResource", "requestKind", "requestResource", "requestSubResource", "name",
               "namespace", "operation", "userInfo", "object", "oldObject", "dryRun", "options")
_GVK, _GVR = ("group", "version", "kind"), ("group", "version", "resource")


def _dup_field(obj, fields):
    seen = set()
    for k, _ in obj:
        if k in fields:
            if k in seen:
                return True
            seen.add(k)
    return False


def _loads_pairs(text):
    return json.loads(text, object_pairs_hook=_Obj)


_AA_PREFIX = "container.apparmor.security.beta.kubernetes.io/"
# include/kwgpu.h KW_CTR_* / KW_REQ_*
_CTR_PRIVILEGED, _CTR_INIT, _CTR_EPHEMERAL, _CTR_HAS_IMAGE, _CTR_HAS_APPARMOR = 1, 2, 4, 8, 16
_REQ_RAW, _REQ_HAS_NAMESPACE, _REQ_HAS_PODSPEC, _REQ_HAS_OBJECT = 1, 2, 4, 8


def flatten_doc(text, raw=False):
    """The columns of one AdmissionReview / RawReview body (the extraction rules of
    SURVEY a15/a16), restated from the JSON value itself, independently of the product's parser:
    {"flags", "uid", "ns", "op", "kind", "containers": [(flags, name, image, aa, adds, drops)],
    "labels": [(key, value)]}, or None when the body is not a request of that type (the product
    answers 400 / 422; the exact rejection texts are pinned elsewhere)."""
    try:
        d = _loads_pairs(text)
    except (ValueError, RecursionError):
        return None
    if not isinstance(d, _Obj) or d.get("request", _Obj) is _Obj:
        return None
    req = d.get("request")
    is_str = lambda v: isinstance(v, str)
    # serde-derived structs refuse a repeated known field (AdmissionReviewRequest / RawReviewRequest,
    # AdmissionRequest, GroupVersionKind / Resource, UserInfo); serde_json::Value members (object,
    # oldObject, a raw request) keep the last one
    if _dup_field(d, ("request",) if raw else ("request", "kind", "apiVersion")):
        return None
    if not raw and isinstance(req, _Obj):
        if _dup_field(req, _REQ_FIELDS):
            return None
        for k, fields in (("kind", _GVK), ("requestKind", _GVK), ("resource", _GVR), ("requestResource", _GVR),
                          ("userInfo", ("username", "uid", "groups", "extra"))):
            v = req.get(k)
            if isinstance(v, _Obj) and _dup_field(v, fields):
                return None
    if not raw:
        for k in ("kind", "apiVersion"):
            if d.get(k) is not None and not is_str(d.get(k)):
                return None
        if not isinstance(req, _Obj):
            return None
        for k, fields in (("uid", None), ("kind", ("group", "version", "kind")), ("resource", ("group", "version", "resource")),
                          ("operation", None)):
            v = req.get(k, _Obj)
            if v is _Obj:
                return None
            if fields is None and not is_str(v):
                return None
            if fields is not None and (not isinstance(v, _Obj) or any(not is_str(v.get(f)) for f in fields)):
                return None
        if not isinstance(req.get("userInfo"), _Obj):
            return None
        for k in ("namespace", "name", "subResource", "requestSubResource"):
            if req.get(k) is not None and not is_str(req.get(k)):
                return None
    r = req if isinstance(req, _Obj) else _Obj()
    sv = lambda v: v if is_str(v) else ""
    flags = _REQ_RAW if raw else 0
    if is_str(r.get("namespace")):
        flags |= _REQ_HAS_NAMESPACE
    rk = r.get("kind")
    rkind = sv(rk.get("kind")) if isinstance(rk, _Obj) else ""
    row = {"uid": sv(r.get("uid")), "ns": sv(r.get("namespace")), "op": sv(r.get("operation")), "kind": rkind,
           "containers": [], "labels": []}
    obj = r.get("object")

    def walk(o, keys):
        for k in keys:
            if not isinstance(o, _Obj):
                return None
            o = o.get(k)
        return o
    if isinstance(obj, _Obj):
        flags |= _REQ_HAS_OBJECT
        kind = obj.get("kind") if is_str(obj.get("kind")) else rkind
        spec = meta = None
        if kind == "Pod":
            spec, meta = obj.get("spec"), obj.get("metadata")
        elif kind in _WORKLOADS:
            spec, meta = walk(obj, ["spec", "template", "spec"]), walk(obj, ["spec", "template", "metadata"])
        elif kind == "CronJob":
            spec = walk(obj, ["spec", "jobTemplate", "spec", "template", "spec"])
            meta = walk(obj, ["spec", "jobTemplate", "spec", "template", "metadata"])
        if isinstance(spec, _Obj):
            flags |= _REQ_HAS_PODSPEC
            ann = meta.get("annotations") if isinstance(meta, _Obj) else None
            for lst, kf in (("containers", 0), ("initContainers", _CTR_INIT), ("ephemeralContainers", _CTR_EPHEMERAL)):
                items = spec.get(lst)
                if not isinstance(items, list) or isinstance(items, _Obj):
                    continue
                for c in items:
                    if not isinstance(c, _Obj):
                        continue
                    cf = kf
                    name, image = sv(c.get("name")), c.get("image")
                    if is_str(image):
                        cf |= _CTR_HAS_IMAGE
                    sc = c.get("securityContext")
                    if isinstance(sc, _Obj) and sc.get("privileged") is True:
                        cf |= _CTR_PRIVILEGED
                    caps = sc.get("capabilities") if isinstance(sc, _Obj) else None

                    def cap_list(k):
                        v = caps.get(k) if isinstance(caps, _Obj) else None
                        return [x for x in v if is_str(x)] if isinstance(v, list) and not isinstance(v, _Obj) else []
                    profile = ""
                    if isinstance(ann, _Obj):
                        for k, v in ann:
                            if k == _AA_PREFIX + name and is_str(v):
                                profile = v
                                cf |= _CTR_HAS_APPARMOR
                    row["containers"].append((cf, name, sv(image), profile, cap_list("add"), cap_list("drop")))
        labels = walk(obj, ["metadata", "labels"])
        if isinstance(labels, _Obj):
            row["labels"] = [(k, v) for k, v in labels if is_str(v)]
    row["flags"] = flags
    return row


def capabilities_patch(required_drops, default_adds, doc):
    """RFC 6902 ops of the psp-capabilities mutation: per container of containers,
    initContainers, ephemeralContainers (JSON array index), the required drops it does not drop
    (none when it drops ALL) and the default adds it neither adds nor drops, settings order; added
    as a new securityContext / capabilities object / list where absent, else appended ("-")."""
    def uniq(xs):
        out = []
        for x in xs:
            if x not in out:
                out.append(x)
        return out
    reqd, defa = uniq(required_drops), uniq(default_adds)
    spec, ptr = podspec(json.loads(doc))
    ops = []
    if spec is None:
        return ops
    for ln in ("containers", "initContainers", "ephemeralContainers"):
        arr = spec.get(ln)
        if not isinstance(arr, list):
            continue
        for k, c in enumerate(arr):
            if not isinstance(c, dict):
                continue
            sc = c.get("securityContext")
            caps = sc.get("capabilities") if isinstance(sc, dict) else None
            add = caps.get("add") if isinstance(caps, dict) else None
            drop = caps.get("drop") if isinstance(caps, dict) else None
            has = lambda lst, x: isinstance(lst, list) and any(isinstance(e, str) and e == x for e in lst)
            mdrop = [] if has(drop, "ALL") else [x for x in reqd if not has(drop, x)]
            madd = [x for x in defa if not has(add, x) and not has(drop, x)]
            if not mdrop and not madd:
                continue
            base = f"{ptr}/{ln}/{k}/securityContext"
            capobj = {}
            if madd:
                capobj["add"] = madd
            if mdrop:
                capobj["drop"] = mdrop
            if not isinstance(sc, dict):
                ops.append({"op": "add", "path": base, "value": {"capabilities": capobj}})
            elif not isinstance(caps, dict):
                ops.append({"op": "add", "path": base + "/capabilities", "value": capobj})
            else:
                for name, lst, cur in (("add", madd, add), ("drop", mdrop, drop)):
                    if not lst:
                        continue
                    if not isinstance(cur, list):
                        ops.append({"op": "add", "path": f"{base}/capabilities/{name}", "value": lst})
                    else:
                        ops.extend({"op": "add", "path": f"{base}/capabilities/{name}/-", "value": x} for x in lst)
    return ops


# ----------------------------------------------------------------------------- PolicyID
class InvalidPolicyId(Exception):
    pass


def parse_policy_id(s):
    """policy_id.rs:29-47 -> ("policy", name) | ("member", group, name)."""
    if s == "":
        raise InvalidPolicyId("Not a valid Policy ID: ")
    parts = s.split("/")
    if len(parts) == 1:
        return ("policy", s)
    if len(parts) == 2:
        return ("member", parts[0], parts[1])
    raise InvalidPolicyId(f"Not a valid Policy ID: {s}")


def policy_id_display(pid):
    return pid[1] if pid[0] == "policy" else f"{pid[1]}/{pid[2]}"


# ----------------------------------------------------------------------------- constraints
def constraints(policy_id, mode, allowed_to_mutate, resp):
    """validation_response_with_constraints (service.rs:160-208) on a response dict."""
    resp = dict(resp)
    if mode == PROTECT:
        if resp.get("patch") is not None and not allowed_to_mutate:
            resp["allowed"] = False
            resp["status"] = {"message": f"Request rejected by policy {policy_id}. The policy attempted to mutate "
                                         f"the request, but it is currently configured to not allow mutations."}
            resp.pop("patch", None)
            resp.pop("patchType", None)
        return resp
    resp["allowed"] = True
    for k in ("patch", "patchType", "status"):
        resp.pop(k, None)
    return resp


def service_evaluate(policy_id, mode, allowed_to_mutate, origin, vanilla, uid, namespace=None, always_accept=None,
                     raw=False, init_error=None):
    """service::evaluate (service.rs:30-152) over a given vanilla response (the reference's mocked
    EvaluationEnvironment, service.rs:224-283)."""
    if not raw and namespace is not None and always_accept is not None and namespace == always_accept:
        return {"uid": uid, "allowed": True}
    if init_error is not None:
        return {"uid": uid, "allowed": False, "status": {"message": init_error, "code": 500}}
    resp = dict(vanilla)
    resp["uid"] = uid
    if origin == VALIDATE:
        resp = constraints(policy_id, mode, allowed_to_mutate, resp)
    return resp


# ----------------------------------------------------------------------------- schema
class ConfigError(Exception):
    pass


def _is_str_list(v):
    return isinstance(v, list) and all(isinstance(x, str) for x in v)


def _family(module):
    for key, fam in (("pod-privileged", F_PRIV), ("namespace-validate", F_NS), ("trusted-repos", F_TRUSTED),
                     ("psp-capabilities", F_CAPS), ("psp-apparmor", F_AA), ("safe-labels", F_LABELS)):
        if key in module:
            return fam
    return 0


_ABSENT = object()


def _ctx_ok(v):
    """`#[serde(default)] context_aware_resources: BTreeSet<_>` (config.rs:349-350, 376-378): an
    absent key is the empty set; an explicit null is not a sequence and fails the variant."""
    if v is _ABSENT:
        return True
    return isinstance(v, list) and all(isinstance(x, dict) and isinstance(x.get("apiVersion"), str)
                                       and isinstance(x.get("kind"), str) for x in v)


def _mode(v):
    """`#[serde(default)] policy_mode: PolicyMode` (config.rs:287-294, 369-371): absent -> Protect;
    present -> serde's buffered enum form: the variant name as a string, or a one-key map whose
    value is unit ({"protect": null}). An explicit null matches neither."""
    if v is _ABSENT:
        return PROTECT
    if isinstance(v, dict) and len(v) == 1:
        (k, val), = v.items()
        if val is None:
            v = k
    if v == "protect":
        return PROTECT
    if v == "monitor":
        return MONITOR
    raise ValueError(v)


def parse_entry(name, v):
    """Untagged PolicyOrPolicyGroup (config.rs:360-394)."""
    if isinstance(v, dict):
        try:
            if isinstance(v.get("module"), str):
                mode = _mode(v.get("policyMode", _ABSENT))
                a2m = v.get("allowedToMutate")
                if a2m is not None and not isinstance(a2m, bool):
                    raise ValueError
                st = v.get("settings")
                if st is not None and not isinstance(st, dict):
                    raise ValueError
                if not _ctx_ok(v.get("contextAwareResources", _ABSENT)):
                    raise ValueError
                return {"name": name, "group": False, "module": v["module"], "mode": mode, "a2m": bool(a2m),
                        "settings": st or {}}
        except ValueError:
            pass
        try:
            mode = _mode(v.get("policyMode", _ABSENT))
            pols, ex, msg = v.get("policies"), v.get("expression"), v.get("message")
            if isinstance(pols, dict) and isinstance(ex, str) and isinstance(msg, str):
                members = []
                for mn, mv in pols.items():
                    if not isinstance(mv, dict) or set(mv) - {"module", "settings", "contextAwareResources"}:
                        raise ValueError
                    if not isinstance(mv.get("module"), str):
                        raise ValueError
                    if mv.get("settings") is not None and not isinstance(mv.get("settings"), dict):
                        raise ValueError
                    if not _ctx_ok(mv.get("contextAwareResources", _ABSENT)):
                        raise ValueError
                    members.append({"name": mn, "module": mv["module"], "settings": mv.get("settings") or {}})
                return {"name": name, "group": True, "mode": mode, "expression": ex, "message": msg,
                        "members": members}
        except ValueError:
            pass
    raise ConfigError("data did not match any variant of untagged enum PolicyOrPolicyGroup")


def validate_policies(entries):
    """config.rs:237-258"""
    for e in entries:
        if "/" in e["name"]:
            raise ConfigError(f"policy name '{e['name']}' contains a '/' character")
        if e["group"]:
            bad = [m["name"] for m in e["members"] if "/" in m["name"]]
            if bad:
                raise ConfigError(f"policy group '{e['name']}' contains policies with invalid names: "
                                  + "[" + ", ".join(f'"{b}"' for b in bad) + "]")


# ----------------------------------------------------------------------------- settings
def compile_settings(fam, s, olib):
    """Returns (lists[5], flags) or raises ValueError(message) -> 'Policy settings are invalid: ...'."""
    L = [[], [], [], [], []]
    flags = 0

    def lst(obj, key, path):
        if obj is None:
            return []
        v = obj.get(key)
        if v is None:
            return []
        if not _is_str_list(v):
            raise ValueError(f"{path} must be a list of strings")
        return list(v)

    def obj_of(key, path):
        v = s.get(key)
        if v is None:
            return None
        if not isinstance(v, dict):
            raise ValueError(f"{path} must be a mapping")
        return v

    if fam == F_PRIV:
        for k, bit in (("skip_init_containers", 1), ("skip_ephemeral_containers", 2)):
            v = s.get(k)
            if v is None:
                continue
            if not isinstance(v, bool):
                raise ValueError(f"{k} must be a boolean")
            if v:
                flags |= bit
    elif fam == F_NS:
        v = s.get("valid_namespace")
        if not isinstance(v, str) or v == "":
            raise ValueError("valid_namespace must be a non-empty string")
        L[0] = [v]
    elif fam == F_TRUSTED:
        reg, tags, imgs = obj_of("registries", "registries"), obj_of("tags", "tags"), obj_of("images", "images")
        L[0], L[1] = lst(reg, "allow", "registries.allow"), lst(reg, "reject", "registries.reject")
        L[2] = lst(tags, "reject", "tags.reject")
        L[3], L[4] = lst(imgs, "allow", "images.allow"), lst(imgs, "reject", "images.reject")
        if L[0] and L[1]:
            raise ValueError("registries: allow and reject lists are mutually exclusive")
        if L[3] and L[4]:
            raise ValueError("images: allow and reject lists are mutually exclusive")
        for g in L[0] + L[1] + L[2] + L[3] + L[4]:
            if not olib.orc_glob_ok(g.encode()):
                raise ValueError(f"invalid pattern '{g}'")
    elif fam == F_CAPS:
        L[0] = lst(s, "allowed_capabilities", "allowed_capabilities")
        L[1] = lst(s, "required_drop_capabilities", "required_drop_capabilities")
        L[2] = lst(s, "default_add_capabilities", "default_add_capabilities")
        if "*" in L[0]:
            flags |= 4
        overlap = [c for c in L[2] if c in L[1]]
        if overlap:
            raise ValueError("these capabilities cannot be both added by default and required to be dropped: "
                             + ", ".join(overlap))
    elif fam == F_AA:
        L[0] = lst(s, "allowed_profiles", "allowed_profiles")
    elif fam == F_LABELS:
        L[0] = lst(s, "denied_labels", "denied_labels")
        L[1] = lst(s, "mandatory_labels", "mandatory_labels")
        c = obj_of("constrained_labels", "constrained_labels")
        for k, v in (c or {}).items():
            if not isinstance(v, str):
                raise ValueError("constrained_labels values must be strings")
            if not olib.orc_regex_ok(v.encode()):
                raise ValueError(f"constrained label '{k}' has an invalid regular expression")
            L[2].append(k)
            L[3].append(v)
        for k in L[0]:
            if k in L[1] or k in L[2]:
                raise ValueError(f"label '{k}' cannot be both denied and mandatory or constrained")
    return L, flags


# ----------------------------------------------------------------------------- group expressions
# The rhai subset of policy-group expressions lives in oracle/rhaisub.py (its own tokenizer, parser
# and evaluator, independent of the product's expr.cpp). Validation runs the script with every
# member returning true; evaluation needs a bool.
ExprError = rhaisub.ExprError
_I64 = (rhaisub.I64_MIN, rhaisub.I64_MAX)


def parse_script(s, members):
    """Script -> rhaisub.Program (raises ExprError on a syntax error or a refused construct)."""
    return rhaisub.parse(s, list(members))


def run_script(prog, members, member_ok):
    """-> (error message or None, bool value, called members in call order)."""
    err, v, called, _ = rhaisub.run(prog, list(members), member_ok)
    return err, v, called


def group_eval_message(m):
    if m.startswith("Output type incorrect"):
        return "policy group expression did not evaluate to a boolean: " + m
    return "policy group expression evaluation failed: " + m


def parse_expression(s, members):
    """The group expression as the bool-only tree the C restatement evaluates (rhaisub.bool_tree);
    raises ExprError when the script does not validate or is not bool-only."""
    members = list(members)
    prog = rhaisub.parse(s, members)
    err, _, _, _ = rhaisub.run(prog, members, [True] * len(members))
    if err is not None and not err.startswith("Output type incorrect"):
        raise ExprError(err)
    t = rhaisub.bool_tree(prog, members)
    if t is None:
        raise ExprError("not a bool-only expression")
    return t


def expr_depth(n, d=1):
    """Max value-stack depth of the short-circuit jump code (same bound as the product: || and &&
    pop their left side before the right one runs; == and != keep it)."""
    if n[0] in ("const", "call"):
        return d
    if n[0] == "not":
        return expr_depth(n[1], d)
    if n[0] in ("and", "or"):
        return max(expr_depth(n[1], d), expr_depth(n[2], d))
    return max(expr_depth(n[1], d), expr_depth(n[2], d + 1))


def eval_expression(n, member_ok):
    """Short-circuit evaluation of a bool-only tree -> (value, called-members list in call order)."""
    called = []

    def ev(x):
        k = x[0]
        if k == "const":
            return bool(x[2])
        if k == "call":
            if x[1] not in called:
                called.append(x[1])
            return member_ok[x[1]]
        if k == "not":
            return not ev(x[1])
        if k == "and":
            return ev(x[1]) and ev(x[2])
        if k == "or":
            return ev(x[1]) or ev(x[2])
        a = ev(x[1])
        b = ev(x[2])
        return (a == b) if k == "eq" else (a != b)

    return ev(n), called


def _to_nodes(root):
    nodes = []

    def emit(x):
        k = x[0]
        if k == "const":
            nodes.append((X_CONST, 1 if x[2] else 0, 0))
        elif k == "call":
            nodes.append((X_CALL, x[1], 0))
        elif k == "not":
            a = emit(x[1])
            nodes.append((X_NOT, a, 0))
        else:
            a = emit(x[1])
            b = emit(x[2])
            nodes.append(({"and": X_AND, "or": X_OR, "eq": X_EQ, "ne": X_NE}[k], a, b))
        return len(nodes) - 1

    emit(root)
    return nodes


# ----------------------------------------------------------------------------- ctypes
class _Strcol(C.Structure):
    _fields_ = [("off", C.POINTER(C.c_uint32)), ("bytes", C.POINTER(C.c_uint8)), ("n", C.c_uint64)]


class Soa(C.Structure):
    """kw_soa layout (include/kwgpu.h)."""
    _fields_ = [
        ("n_requests", C.c_uint64), ("req_flags", C.POINTER(C.c_uint8)), ("ctr_off", C.POINTER(C.c_uint32)),
        ("lbl_off", C.POINTER(C.c_uint32)), ("uid", _Strcol), ("ns", _Strcol), ("op", _Strcol), ("kind", _Strcol),
        ("ctr_flags", C.POINTER(C.c_uint8)), ("capadd_off", C.POINTER(C.c_uint32)),
        ("capdrop_off", C.POINTER(C.c_uint32)), ("ctr_name", _Strcol), ("ctr_image", _Strcol),
        ("ctr_apparmor", _Strcol), ("cap_add", _Strcol), ("cap_drop", _Strcol), ("lbl_key", _Strcol),
        ("lbl_val", _Strcol),
    ]


class _XNode(C.Structure):
    _fields_ = [("op", C.c_int32), ("a", C.c_int32), ("b", C.c_int32)]


class _OPolicy(C.Structure):
    _fields_ = [("family", C.c_int32), ("mode", C.c_int32), ("allowed_to_mutate", C.c_int32),
                ("init_error", C.c_int32), ("expr_error", C.c_int32), ("flags", C.c_int32),
                ("n", C.c_int32 * 5), ("l", C.POINTER(C.c_char_p) * 5), ("n_members", C.c_int32),
                ("members", C.POINTER(C.c_int32)), ("n_nodes", C.c_int32), ("nodes", C.POINTER(_XNode)),
                ("table", C.POINTER(C.c_uint32))]


class _ODetail(C.Structure):
    _fields_ = [("word", C.c_uint32), ("reason", C.c_uint32), ("arg", C.c_uint64), ("mutated", C.c_uint32),
                ("bypass", C.c_uint32), ("ncauses", C.c_int32), ("causes", C.c_int32 * 4096)]


_olib = None


def olib():
    global _olib
    if _olib is None:
        L = C.CDLL(LIB)
        L.orc_env_new.restype = C.c_void_p
        L.orc_env_new.argtypes = [C.POINTER(_OPolicy), C.c_int32, C.c_char_p, C.c_char_p, C.c_int]
        L.orc_env_free.argtypes = [C.c_void_p]
        L.orc_eval.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.c_int32, C.c_uint64,
                               C.c_uint64, C.POINTER(C.c_uint32)]
        L.orc_eval_mt.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.c_int32, C.c_uint64,
                                  C.c_int, C.POINTER(C.c_uint32)]
        L.orc_eval_mt_pinned.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.c_int32,
                                         C.c_uint64, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_uint32)]
        L.orc_image_parts.restype = C.c_int
        L.orc_image_parts.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        L.orc_eval_detail.restype = None
        L.orc_eval_detail.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_uint64, C.POINTER(_ODetail)]
        L.orc_regex_ok.restype = C.c_int
        L.orc_regex_ok.argtypes = [C.c_char_p]
        L.orc_re_match.restype = C.c_int
        L.orc_re_match.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        L.orc_glob_ok.restype = C.c_int
        L.orc_glob_ok.argtypes = [C.c_char_p]
        L.orc_glob_match.restype = C.c_int
        L.orc_glob_match.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        _olib = L
    return _olib


def regex_match(pattern, subject):
    """The oracle's Regex::is_match (oracle/kwregex.c): 1 / 0, or -1 when the pattern does not
    compile in the dialect of DESIGN.md §2."""
    b = subject.encode() if isinstance(subject, str) else bytes(subject)
    return olib().orc_re_match(pattern.encode(), b, len(b))


def glob_match(pattern, subject):
    """The oracle's glob match (oracle/kwregex.c, fnmatch(3) flags 0 over code points): 1 / 0, or -1
    when the glob is outside the dialect of DESIGN.md §2."""
    b = subject.encode() if isinstance(subject, str) else bytes(subject)
    return olib().orc_glob_match(pattern.encode(), b, len(b))


def image_parts(image):
    n = len(image.encode()) * 2 + 64
    reg, tag, norm = C.create_string_buffer(n), C.create_string_buffer(n), C.create_string_buffer(n * 2)
    eff = olib().orc_image_parts(image.encode(), reg, tag, norm, len(norm))
    return reg.value.decode(), tag.value.decode() if eff else None, norm.value.decode()


# ----------------------------------------------------------------------------- environment
class OracleEnv:
    """Restated EvaluationEnvironment. Policy order: top-level entries in document order, then group
    members (group order, settings order) — the same order the product uses, checked by tests via ids."""

    def __init__(self, policies, continue_on_errors=False, always_accept_namespace=None):
        L = olib()
        if isinstance(policies, (str, bytes)):
            policies = json.loads(policies)
        entries = [parse_entry(k, v) for k, v in policies.items()]
        validate_policies(entries)
        self.always_ns = always_accept_namespace
        self.pol = []
        for e in entries:
            if e["name"] == "":
                raise InvalidPolicyId("Not a valid Policy ID: ")
            p = {"id": e["name"], "name": e["name"], "group": e["group"], "member": False, "mode": e["mode"],
                 "a2m": False, "registered": True, "init_error": None, "family": F_GROUP if e["group"] else 0,
                 "lists": [[], [], [], [], []], "flags": 0}
            if e["group"]:
                p.update(expression=e["expression"], message=e["message"],
                         member_names=[m["name"] for m in e["members"]], members=[], broken=None)
            else:
                p.update(module=e["module"], a2m=e["a2m"], settings=e["settings"])
            self.pol.append(p)
        for gi, e in enumerate(entries):
            if not e["group"]:
                continue
            for m in e["members"]:
                self.pol[gi]["members"].append(len(self.pol))
                self.pol.append({"id": f"{e['name']}/{m['name']}", "name": m["name"], "group": False,
                                 "member": True, "parent": gi, "mode": PROTECT, "a2m": False, "registered": True,
                                 "init_error": None, "module": m["module"], "settings": m["settings"],
                                 "lists": [[], [], [], [], []], "flags": 0, "family": 0})
        for p in self.pol:
            if p["group"]:
                continue
            fam = _family(p["module"])
            err = None
            if fam == 0:
                p["registered"] = False
                err = (f"bootstrap failure: {p['id']}: policy module '{p['module']}' is not in the declarative "
                       f"policy class served by kwgpu")
            else:
                p["family"] = fam
                try:
                    p["lists"], p["flags"] = compile_settings(fam, p["settings"], L)
                except ValueError as ex:
                    err = f"Policy settings are invalid: {ex}"
            if err is not None:
                if not continue_on_errors:
                    raise ConfigError(err)
                p["init_error"] = err
                if p["member"]:
                    g = self.pol[p["parent"]]
                    if g["broken"] is None:
                        g["broken"] = p["id"]
        for p in self.pol:
            if not p["group"]:
                continue
            p["expr_error"] = None
            p["pyscript"] = False
            p["ast"] = None
            p["script"] = None
            p["table"] = None
            names = p["member_names"]
            try:
                root = parse_script(p["expression"], names)
                # validate_settings: members return true
                err, _, _, steps = rhaisub.run(root, names, [True] * len(names))
                if err is not None and not err.startswith("Output type incorrect"):
                    raise ExprError(err)
                p["valid"] = True
                p["script"] = root
                if not rhaisub.calls_members(root, names):  # one outcome
                    err, v, _ = run_script(root, names, [True] * len(names))
                    if err is not None:
                        p["expr_error"] = group_eval_message(err)
                    else:
                        p["ast"] = ("const", "bool", v)
                    continue
                t = rhaisub.bool_tree(root, names)
                if t is not None:
                    if len(names) > 65535 or expr_depth(t) > 65536:
                        raise ExprError("policy group expression exceeds the engine's limits (65535 members, value "
                                        "stack 65536)")
                    p["ast"] = t
                elif len(names) > 12 or (max(steps, 1) << len(names)) > (1 << 18):
                    p["pyscript"] = True  # run_script per row (_pyscript) instead of a table
                else:  # every vector of member results: value, error, causes (the C half looks it up)
                    tab = []
                    for mask in range(1 << len(names)):
                        ok = [bool((mask >> i) & 1) for i in range(len(names))]
                        err, v, called = run_script(root, names, ok)
                        e = 2 if err is not None else (1 if v else 0)
                        for c in called:
                            if not ok[c]:
                                e |= 1 << (16 + c)
                        tab.append(e)
                    p["table"] = tab
            except ExprError as ex:
                p["expr_error"] = str(ex)
                p["valid"] = False
        self.ids = {p["id"]: i for i, p in enumerate(self.pol)}
        self._build_c()

    def _build_c(self):
        n = len(self.pol)
        self._arr = (_OPolicy * n)()
        self._keep = []
        for i, p in enumerate(self.pol):
            o = self._arr[i]
            o.family = p["family"]
            o.mode = p["mode"]
            o.allowed_to_mutate = 1 if p["a2m"] else 0
            o.init_error = 1 if p["init_error"] else 0
            o.flags = p["flags"]
            for k in range(5):
                items = [s.encode() for s in p["lists"][k]]
                arr = (C.c_char_p * max(len(items), 1))(*items)
                self._keep.append(arr)
                o.n[k] = len(items)
                o.l[k] = C.cast(arr, C.POINTER(C.c_char_p))
            if p["group"]:
                # (a _pyscript group: the C half answers GROUP_EXPR, Python replaces its words)
                o.expr_error = 1 if (p["expr_error"] or p["pyscript"]) else 0
                mem = (C.c_int32 * max(len(p["members"]), 1))(*p["members"])
                self._keep.append(mem)
                o.n_members = len(p["members"])
                o.members = C.cast(mem, C.POINTER(C.c_int32))
                if p["table"] is not None:
                    tab = (C.c_uint32 * len(p["table"]))(*p["table"])
                    self._keep.append(tab)
                    o.table = C.cast(tab, C.POINTER(C.c_uint32))
                if p["ast"] is not None:
                    nodes = _to_nodes(p["ast"])
                    xs = (_XNode * len(nodes))(*[_XNode(*t) for t in nodes])
                    self._keep.append(xs)
                    o.n_nodes = len(nodes)
                    o.nodes = C.cast(xs, C.POINTER(_XNode))
        err = C.create_string_buffer(512)
        self._h = olib().orc_env_new(self._arr, n, self.always_ns.encode() if self.always_ns else None, err, 512)
        if not self._h:
            raise ConfigError("oracle regex compilation failed: " + err.value.decode())

    def __del__(self):
        try:
            olib().orc_env_free(self._h)
        except Exception:
            pass

    def lookup(self, policy_id):
        parse_policy_id(policy_id)
        if policy_id not in self.ids:
            raise KeyError(f"unknown policy: {policy_id}")
        return self.ids[policy_id]

    # ---- groups beyond the bool subset with more than 16 members: the C half has no truth table for
    # them, so their words come from run_script (this file's own interpreter) over the members' own
    # evaluations, composed like kworacle.c detail() composes a group's word
    @staticmethod
    def _group_word(P, reason, mask, origin):
        n = len(P["members"])
        arg16 = 0 if reason != R_GROUP else (0xFFFF if n > 15 else mask)
        v = (reason << 8) | (arg16 << 16)
        allowed = reason == 0
        fst, fallowed = (0 if allowed else 1), allowed
        if origin == VALIDATE and P["mode"] == MONITOR:
            fst, fallowed = 0, True
        if allowed:
            v |= 1  # V_ALLOWED
        if fallowed:
            v |= 4  # F_ALLOWED
        return v | (fst << 3)

    def _pyscript(self, P, member_ok):
        """-> (reason, cause mask, cause slots) of a _pyscript group over its members' results."""
        err, value, called = run_script(P["script"], P["member_names"], member_ok)
        if err is not None:
            return R_GROUP_EXPR, 0, []
        if value:
            return 0, 0, []
        causes = sorted(c for c in called if not member_ok[c])  # slot order, as kworacle.c lists causes
        return R_GROUP, sum(1 << c for c in causes), causes

    def _member_ok(self, P, words):
        return [bool(w & 1) and not (w & 2) for w in words]

    def eval(self, soa, policies, origin=VALIDATE, rows=None, threads=1, cpus=None):
        """Verdict words for rows x policies (numpy uint32, row-major); cpus: pin thread t to CPU
        cpus[t]."""
        idx = [self.lookup(p) if isinstance(p, str) else p for p in policies]
        out = self._eval_c(soa, idx, origin, rows, threads, cpus)
        py = [j for j, i in enumerate(idx) if self.pol[i]["group"] and self.pol[i].get("pyscript")]
        if py:
            n = soa.n_requests if rows is None else rows
            w = out.reshape(n, len(idx))
            for j in py:
                P = self.pol[idx[j]]
                mw = self._eval_c(soa, P["members"], origin, rows, threads, cpus).reshape(n, len(P["members"]))
                for r in range(n):
                    if w[r, j] & 0x20:  # the namespace bypass word stays
                        continue
                    reason, mask, _ = self._pyscript(P, self._member_ok(P, mw[r]))
                    w[r, j] = self._group_word(P, reason, mask, origin)
        return out

    def _eval_c(self, soa, idx, origin, rows, threads, cpus):
        n = soa.n_requests if rows is None else rows
        arr = (C.c_int32 * len(idx))(*idx)
        out = np.zeros(n * len(idx), dtype=np.uint32)
        ptr = out.ctypes.data_as(C.POINTER(C.c_uint32))
        if cpus is not None:
            pin = (C.c_int32 * len(cpus))(*cpus)
            olib().orc_eval_mt_pinned(self._h, C.byref(soa), arr, len(idx), origin, n, len(cpus), pin, ptr)
        elif threads > 1:
            olib().orc_eval_mt(self._h, C.byref(soa), arr, len(idx), origin, n, threads, ptr)
        else:
            olib().orc_eval(self._h, C.byref(soa), arr, len(idx), origin, 0, n, ptr)
        return out

    # ------------------------------------------------------------------ responses
    def message(self, soa, row, pidx, reason, arg):
        """Message templates (DESIGN.md §Policy families)."""
        P = self.pol[pidx]

        def s(col, i):
            c = getattr(soa, col)
            return bytes(c.bytes[c.off[i]:c.off[i + 1]]).decode()

        cb, lb = soa.ctr_off[row], soa.lbl_off[row]
        q = lambda x: f"'{x}'"  # noqa: E731
        if reason == R_PRIVILEGED:
            return "Privileged container is not allowed"
        if reason == R_NAMESPACE:
            return f"namespace {q(s('ns', row))} is not accepted: only {q(P['lists'][0][0])} is allowed"
        if reason in (R_REG_NOT_ALLOWED, R_REG_REJECTED, R_TAG_REJECTED, R_IMG_NOT_ALLOWED, R_IMG_REJECTED):
            image = s("ctr_image", cb + arg)
            reg, tag, _ = image_parts(image)
            head = f"container {q(s('ctr_name', cb + arg))} uses image {q(image)}"
            return {R_REG_NOT_ALLOWED: f"{head}: registry {q(reg)} is not in the allowed registries",
                    R_REG_REJECTED: f"{head}: registry {q(reg)} is rejected",
                    R_TAG_REJECTED: f"{head}: tag {q(tag)} is rejected",
                    R_IMG_NOT_ALLOWED: f"{head}, which is not in the allowed images",
                    R_IMG_REJECTED: f"{head}, which is rejected"}[reason]
        if reason == R_CAP:  # arg: index in the request's add lists, flattened in container order
            k = soa.capadd_off[cb] + arg
            c = cb
            while soa.capadd_off[c + 1] <= k:
                c += 1
            return f"container {q(s('ctr_name', c))} adds capability {q(s('cap_add', k))}, which is not allowed"
        if reason == R_APPARMOR:
            return (f"container {q(s('ctr_name', cb + arg))} uses AppArmor profile "
                    f"{q(s('ctr_apparmor', cb + arg))}, which is not allowed")
        if reason == R_LABEL_DENIED:
            return f"label {q(s('lbl_key', lb + arg))} is denied"
        if reason == R_LABEL_CONSTRAINT:  # arg: label index; the constraint is the policy's on its key
            key = s("lbl_key", lb + arg)
            regex = P["lists"][3][P["lists"][2].index(key)]
            return (f"label {q(key)} value {q(s('lbl_val', lb + arg))} does not match the "
                    f"constraint {q(regex)}")
        if reason == R_LABEL_MANDATORY:
            return f"mandatory label {q(P['lists'][1][arg])} is missing"
        if reason == R_GROUP:
            return P["message"]
        if reason == R_GROUP_EXPR:
            if P["expr_error"]:
                return P["expr_error"]
            # a data-dependent evaluation error: the script over this row's member results
            ok = []
            for m in P["members"]:
                md = self.detail(soa, row, m)
                ok.append(md["reason"] == 0 and not md["mutated"])
            err, _, _ = run_script(P["script"], P["member_names"], ok)
            return group_eval_message(err)
        if reason == R_INIT:
            return P["init_error"]
        return ""

    def detail(self, soa, row, pidx, origin=VALIDATE):
        """The oracle's own evaluation of (row, policy): dict(word, reason, arg (full), mutated,
        bypass, causes (member slots))."""
        d = _ODetail()
        olib().orc_eval_detail(self._h, C.byref(soa), pidx, origin, row, C.byref(d))
        out = {"word": d.word, "reason": d.reason, "arg": d.arg, "mutated": bool(d.mutated), "bypass": bool(d.bypass),
               "causes": list(d.causes[:d.ncauses])}
        P = self.pol[pidx]
        if P["group"] and P.get("pyscript") and not out["bypass"]:
            ok = []
            for m in P["members"]:
                md = self.detail(soa, row, m, origin)
                ok.append(md["reason"] == 0 and not md["mutated"])
            reason, mask, causes = self._pyscript(P, ok)
            out.update(word=self._group_word(P, reason, mask, origin), reason=reason, arg=mask, causes=causes)
        return out

    def response_doc(self, soa, row, pidx, origin=VALIDATE, doc=None):
        """AdmissionResponse dict of (row, policy) derived from the oracle's own evaluation of the
        document (service.rs:30-152, 160-208) — independent of any verdict word: full entity
        indices, the group's own short-circuit causes and each cause member's own evaluation.
        Raises KeyError for PolicyNotFound outcomes."""
        P = self.pol[pidx]
        c = soa.uid
        uid = bytes(c.bytes[c.off[row]:c.off[row + 1]]).decode()
        d = self.detail(soa, row, pidx, origin)
        if d["bypass"]:
            if not P["registered"]:
                raise KeyError(f"unknown policy: {P['id']}")
            return {"uid": uid, "allowed": True}
        if P["group"] and P["broken"]:
            raise KeyError(f"unknown policy: {P['broken']}")
        if P["init_error"]:
            return {"uid": uid, "allowed": False, "status": {"message": P["init_error"], "code": 500}}
        reason = d["reason"]
        vanilla = {"uid": uid, "allowed": reason == 0}
        if reason:
            st = {"message": self.message(soa, row, pidx, reason, d["arg"])}
            if reason == R_GROUP_EXPR:
                st["code"] = 500
            if reason == R_GROUP:
                causes = []
                for slot in d["causes"]:
                    m = P["members"][slot]
                    md = self.detail(soa, row, m, origin)
                    if md["reason"] == 0 and md["mutated"]:
                        msg = "mutation is not allowed inside of policy group"
                    else:
                        msg = self.message(soa, row, m, md["reason"], md["arg"])
                    causes.append({"field": f"spec.policies.{self.pol[m]['name']}", "message": msg})
                st["details"] = {"causes": causes}
            vanilla["status"] = st
        elif d["mutated"]:
            if doc is None:
                raise ValueError("the original document is required to restate a mutation")
            ops = capabilities_patch(P["lists"][1], P["lists"][2], doc)
            vanilla["patchType"] = "JSONPatch"
            vanilla["patch"] = base64.b64encode(json.dumps(ops, separators=(",", ":"), ensure_ascii=False).encode()).decode()
        if origin == VALIDATE:
            return constraints(P["id"], P["mode"], P["a2m"], vanilla)
        return vanilla

    def response(self, soa, row, pidx, v, member_v=None, doc=None, wide=None):
        """AdmissionResponse dict the service returns for verdict word v (service.rs:30-152).
        doc: the row's original JSON text, needed for an accepted mutation (the patch); wide(pidx):
        the full argument of a word whose ARG is KW_ARG_WIDE."""
        P = self.pol[pidx]
        c = soa.uid
        uid = bytes(c.bytes[c.off[row]:c.off[row + 1]]).decode()
        if v & 0x20:
            if not P["registered"]:
                raise KeyError(f"unknown policy: {P['id']}")
            return {"uid": uid, "allowed": True}
        if P["group"] and P["broken"]:
            raise KeyError(f"unknown policy: {P['broken']}")
        if v & 0x40:  # F_PATCH: accepted mutation, the response carries the JSONPatch
            if doc is None:
                raise ValueError("the original document is required to restate a mutation")
            ops = capabilities_patch(P["lists"][1], P["lists"][2], doc)
            patch = base64.b64encode(json.dumps(ops, separators=(",", ":"), ensure_ascii=False).encode()).decode()
            return {"uid": uid, "allowed": True, "patchType": "JSONPatch", "patch": patch}
        fst = (v >> 3) & 3
        reason, arg = (v >> 8) & 0xFF, v >> 16
        if arg == 0xFFFF and wide is not None:
            arg = wide(pidx)
        resp = {"uid": uid, "allowed": bool(v & 4)}
        if fst == 0:
            return resp
        if fst == 3:
            resp["status"] = {"message": P["init_error"], "code": 500}
            return resp
        if fst == 2:
            resp["status"] = {"message": f"Request rejected by policy {P['id']}. The policy attempted to mutate the "
                                         f"request, but it is currently configured to not allow mutations."}
            return resp
        st = {"message": self.message(soa, row, pidx, reason, arg)}
        if reason == R_GROUP_EXPR:
            st["code"] = 500
        if reason == R_GROUP:
            causes = []
            for slot, m in enumerate(P["members"]):
                if not (arg >> slot) & 1:
                    continue
                mv = member_v[slot]
                if (mv & 2) and (mv & 1):
                    msg = "mutation is not allowed inside of policy group"
                else:
                    marg = mv >> 16
                    if marg == 0xFFFF and wide is not None:
                        marg = wide(m)
                    msg = self.message(soa, row, m, (mv >> 8) & 0xFF, marg)
                causes.append({"field": f"spec.policies.{self.pol[m]['name']}", "message": msg})
            st["details"] = {"causes": causes}
        resp["status"] = st
        return resp
