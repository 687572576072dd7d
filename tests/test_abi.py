"""CPU: libkwgpu.so loads and exports every entry point declared in include/kwgpu.h; host-only
calls behave; the hot path refuses to run without a device (no silent CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import kwgpu as K
from helpers import ROOT, config, reference_doc


def header_functions():
    text = open(os.path.join(ROOT, "include", "kwgpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kw_[a-z_]+)\s*\(", text)) - {"kw_env_options"})


def test_library_exports_every_header_symbol():
    lib_path = os.path.join(ROOT, "policy-server_amd", "libkwgpu.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (kw_\w+)", out))
    declared = header_functions()
    assert declared, "no functions parsed from include/kwgpu.h"
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    lib = C.CDLL(lib_path)
    for f in declared:
        assert getattr(lib, f)


def test_binding_declares_every_export():
    assert sorted(K._native.EXPORTS) == header_functions()


def test_version_and_gfx950_code_object():
    assert K.library().kw_version().decode().startswith("kwgpu")
    lib_path = os.path.join(ROOT, "policy-server_amd", "libkwgpu.so")
    blob = open(lib_path, "rb").read()
    assert b"gfx950" in blob


def test_hot_path_requires_a_device():
    env = K.EvaluationEnvironment(config("parity"), continue_on_errors=True)  # host-only env
    with pytest.raises(K.DeviceError):
        env.evaluate("pod-privileged", reference_doc("pod_with_privileged_containers.json"))
    b = K.Batch.from_json([reference_doc("pod_with_privileged_containers.json")])
    with pytest.raises(K.EvaluationError):
        b.validate(env, ["pod-privileged"])  # not resident, no device


def test_pin_host_arguments():
    """kw_batch_pin_host refuses a null batch and a negative device (KW_E_ARG) before touching
    the runtime; on a host without a GPU a real device index fails as a device error."""
    L = K._native.lib()
    assert L.kw_batch_pin_host(None, 0) == K._native.KW_E_ARG
    b = K.Batch.from_json([reference_doc("pod_with_privileged_containers.json")])
    with pytest.raises(K.EvaluationError) as e:
        b.pin_host(-1)
    assert e.value.code == K._native.KW_E_ARG
    import torch
    if not torch.cuda.is_available():
        with pytest.raises(K.DeviceError):
            b.pin_host(0)


def test_lookup_and_accessors():
    env = K.EvaluationEnvironment(config("parity"), continue_on_errors=True, always_accept_namespace="kubewarden")
    assert env.get_policy_mode("trusted-images") == K.MONITOR
    assert env.get_policy_mode("pod-privileged") == K.PROTECT
    assert env.get_policy_allowed_to_mutate("psp-capabilities") is False
    assert env.get_policy_mode("group-or/reg") == K.PROTECT  # members always Protect
    assert env.is_group(env.lookup("group-or"))
    assert [env.policy_id(i) for i in env.group_members(env.lookup("group-or"))] == \
        ["group-or/priv", "group-or/reg", "group-or/latest"]
    assert env.should_always_accept_requests_made_inside_of_namespace("kubewarden")
    assert not env.should_always_accept_requests_made_inside_of_namespace("kubewarden-approved")
    # unsupported module: not registered -> mode lookups fail like PolicyNotFound
    with pytest.raises(K.PolicyNotFound):
        env.get_policy_mode("unsupported")
    assert env.policy_initialization_error("bad-settings").startswith("Policy settings are invalid:")
    assert env.policy_initialization_error("unsupported").startswith("bootstrap failure: unsupported:")


def test_serialize_roundtrip():
    env = K.EvaluationEnvironment(config("c4_64"))
    blob = env.serialize()
    env2 = K.EvaluationEnvironment.from_serialized(blob)
    assert env2.policy_ids() == env.policy_ids()
    assert env2.serialize() == blob
    bad = bytearray(blob)
    bad[-20] ^= 0xFF  # corrupt the compiled tables
    with pytest.raises(K.EvaluationError):
        K.EvaluationEnvironment.from_serialized(bytes(bad))
