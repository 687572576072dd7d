"""kwgpu — Python binding of the MI355X admission-evaluation engine (libkwgpu.so).

Plumbing for tests and the benchmark over the C ABI in include/kwgpu.h. Names mirror the
reference so tests read like its own:

  EvaluationEnvironment   src/evaluation/evaluation_environment.rs:86-127 (+ builder :130-366)
  EvaluationError & co    src/evaluation/errors.rs:5-24
  evaluate / RequestOrigin  src/api/service.rs:16-152
  PolicyMode              src/config.rs:287-294

Every evaluation runs on the GPU through the C ABI; nothing here computes a verdict.
"""
import ctypes as C
import json

from . import _native as N
from ._native import KwSoa, KwTiming  # noqa: F401

PROTECT, MONITOR = N.KW_MODE_PROTECT, N.KW_MODE_MONITOR
VALIDATE, AUDIT = N.KW_ORIGIN_VALIDATE, N.KW_ORIGIN_AUDIT


class RequestOrigin:
    Validate = N.KW_ORIGIN_VALIDATE
    Audit = N.KW_ORIGIN_AUDIT


class PolicyMode:
    Protect = N.KW_MODE_PROTECT
    Monitor = N.KW_MODE_MONITOR


class EvaluationError(Exception):
    """errors.rs:5-24; `code` is the KW_E_* status, str() the reference Display string."""

    code = None

    def __init__(self, message, code=None):
        super().__init__(message)
        if code is not None:
            self.code = code


class InvalidPolicyId(EvaluationError):
    code = N.KW_E_INVALID_ID


class PolicyInitialization(EvaluationError):
    code = N.KW_E_INIT


class PolicyNotFound(EvaluationError):
    code = N.KW_E_NOT_FOUND


class BootstrapFailure(EvaluationError):
    code = N.KW_E_BOOTSTRAP


class EngineError(EvaluationError):
    code = N.KW_E_ENGINE


class PayloadError(EvaluationError):
    """HTTP 422 of JsonExtractor (handlers.rs:29-39)."""

    code = N.KW_E_PAYLOAD


class DeviceError(EvaluationError):
    code = N.KW_E_DEVICE


_ERRORS = {c.code: c for c in (InvalidPolicyId, PolicyInitialization, PolicyNotFound, BootstrapFailure,
                               EngineError, PayloadError, DeviceError)}


def raise_for(code, message):
    if code == N.KW_OK:
        return
    cls = _ERRORS.get(code, EvaluationError)
    raise cls(message, code)


def http_status(code):
    """handle_evaluation_error (handlers.rs:321-342) + the 422 of the JSON extractor."""
    if code == N.KW_OK:
        return 200
    if code == N.KW_E_NOT_FOUND:
        return 404
    if code == N.KW_E_PAYLOAD:
        return 422
    return 500


def library():
    return N.lib()


class EvaluationEnvironment:
    """Immutable compiled policy set (EvaluationEnvironmentBuilder::build)."""

    def __init__(self, policies, continue_on_errors=False, always_accept_namespace=None, device=-1, yaml=False):
        """policies: a dict, JSON text, or (yaml=True) the policies.yml text itself."""
        L = N.lib()
        if isinstance(policies, (dict, list)):
            doc = json.dumps(policies).encode()
        elif isinstance(policies, str):
            doc = policies.encode()
        else:
            doc = bytes(policies)
        opts = N.KwEnvOptions(1 if continue_on_errors else 0,
                              always_accept_namespace.encode() if always_accept_namespace is not None else None,
                              device)
        h = C.c_void_p()
        err = C.create_string_buffer(4096)
        build = L.kw_env_build_yaml if yaml else L.kw_env_build
        rc = build(doc, len(doc), C.byref(opts), C.byref(h), err, len(err))
        raise_for(rc, err.value.decode(errors="replace"))
        self._h = h
        self.device = device
        self._L = L

    @classmethod
    def from_serialized(cls, blob, device=-1):
        self = cls.__new__(cls)
        L = N.lib()
        h = C.c_void_p()
        err = C.create_string_buffer(4096)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        rc = L.kw_env_deserialize(buf, len(blob), device, C.byref(h), err, len(err))
        raise_for(rc, err.value.decode(errors="replace"))
        self._h, self.device, self._L = h, device, L
        return self

    def serialize(self):
        need = C.c_size_t()
        self._L.kw_env_serialize(self._h, None, 0, C.byref(need))
        buf = (C.c_uint8 * need.value)()
        rc = self._L.kw_env_serialize(self._h, buf, need.value, C.byref(need))
        raise_for(rc, "serialize")
        return bytes(buf)

    def close(self):
        if getattr(self, "_h", None):
            self._L.kw_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- lookups (evaluation_environment.rs:373-469)
    def lookup(self, policy_id):
        """PolicyID::from_str + map lookup -> policy index; raises InvalidPolicyId / PolicyNotFound."""
        idx = C.c_int32()
        b = policy_id.encode()
        rc = self._L.kw_env_lookup(self._h, b, len(b), C.byref(idx))
        if rc == N.KW_E_INVALID_ID:
            raise InvalidPolicyId(f"Not a valid Policy ID: {policy_id}")
        if rc == N.KW_E_NOT_FOUND:
            raise PolicyNotFound(f"unknown policy: {policy_id}")
        raise_for(rc, policy_id)
        return idx.value

    def policy_count(self):
        return self._L.kw_env_policy_count(self._h)

    def policy_id(self, idx):
        buf = C.create_string_buffer(1024)
        raise_for(self._L.kw_env_policy_id(self._h, idx, buf, len(buf)), "policy_id")
        return buf.value.decode()

    def policy_ids(self):
        return [self.policy_id(i) for i in range(self.policy_count())]

    def is_group(self, idx):
        return self._L.kw_env_is_group(self._h, idx) == 1

    def group_members(self, idx):
        out = (C.c_int32 * 256)()
        n = self._L.kw_env_group_members(self._h, idx, out, 256)
        return list(out[:n])

    def get_policy_mode(self, policy):
        idx = self._idx(policy)
        v = C.c_int()
        rc = self._L.kw_env_get_policy_mode(self._h, idx, C.byref(v))
        if rc == N.KW_E_NOT_FOUND:
            raise PolicyNotFound(f"unknown policy: {self.policy_id(idx)}")
        raise_for(rc, "get_policy_mode")
        return v.value

    def get_policy_allowed_to_mutate(self, policy):
        idx = self._idx(policy)
        v = C.c_int()
        rc = self._L.kw_env_get_policy_allowed_to_mutate(self._h, idx, C.byref(v))
        if rc == N.KW_E_NOT_FOUND:
            raise PolicyNotFound(f"unknown policy: {self.policy_id(idx)}")
        raise_for(rc, "get_policy_allowed_to_mutate")
        return bool(v.value)

    def patterns(self, col):
        """The distinct patterns of request column `col` as (kind, text) (kw_env_pattern)."""
        out = []
        for i in range(self._L.kw_env_pattern_count(self._h, col)):
            kind = C.c_int()
            buf = C.create_string_buffer(1 << 16)
            raise_for(self._L.kw_env_pattern(self._h, col, i, C.byref(kind), buf, len(buf)), "kw_env_pattern")
            out.append((kind.value, buf.value.decode()))
        return out

    def classify(self, col, s, key=b""):
        """Diagnostic (kw_env_classify): the ids of the column patterns `s` matches through the
        compiled classifiers; `key` selects the label key for COL_LV."""
        s = s.encode() if isinstance(s, str) else s
        key = key.encode() if isinstance(key, str) else key
        cap = 4096
        out = (C.c_uint32 * cap)()
        n = self._L.kw_env_classify(self._h, col, key, len(key), s, len(s), out, cap)
        if n < 0:
            raise EngineError("kw_env_classify failed")
        return sorted(out[:min(n, cap)])

    def should_always_accept_requests_made_inside_of_namespace(self, ns):
        b = ns.encode()
        return self._L.kw_env_should_always_accept_requests_made_inside_of_namespace(self._h, b, len(b)) == 1

    def policy_initialization_error(self, policy):
        buf = C.create_string_buffer(4096)
        r = self._L.kw_env_policy_initialization_error(self._h, self._idx(policy), buf, len(buf))
        return buf.value.decode() if r == 1 else None

    def validate_settings(self, policy):
        """Raises like EvaluationEnvironment::validate_settings (evaluation_environment.rs:472-510)."""
        buf = C.create_string_buffer(4096)
        rc = self._L.kw_env_validate_settings(self._h, self._idx(policy), buf, len(buf))
        raise_for(rc, buf.value.decode(errors="replace"))

    def _idx(self, policy):
        return policy if isinstance(policy, int) else self.lookup(policy)

    def _array(self, policies):
        """The policy list as the C ABI's int32 index array, memoised per list: building it costs a
        lookup per policy (~100 us for 64 on the host), more than a small shard's whole pass."""
        key = tuple(policies)
        memo = self.__dict__.setdefault("_arrays", {})
        arr = memo.get(key)
        if arr is None:
            arr = (C.c_int32 * len(policies))(*[self._idx(p) for p in policies])
            if len(memo) > 256:
                memo.clear()
            memo[key] = arr
        return arr

    # --- service::evaluate for one request (service.rs:30-152)
    def evaluate(self, policy_id, document, origin=VALIDATE, raw=False):
        """Returns the AdmissionResponse dict; raises the EvaluationError the handler maps to HTTP."""
        if isinstance(document, (dict, list)):
            document = json.dumps(document)
        doc = document.encode() if isinstance(document, str) else bytes(document)
        need = C.c_size_t()
        buf = C.create_string_buffer(1 << 16)
        rc = self._L.kw_evaluate(self._h, policy_id.encode(), doc, len(doc),
                                 N.KW_DOC_RAW_REVIEW if raw else N.KW_DOC_ADMISSION_REVIEW, origin,
                                 buf, len(buf), C.byref(need))
        if rc == N.KW_E_NOSPACE:
            buf = C.create_string_buffer(need.value)
            rc = self._L.kw_evaluate(self._h, policy_id.encode(), doc, len(doc),
                                     N.KW_DOC_RAW_REVIEW if raw else N.KW_DOC_ADMISSION_REVIEW, origin,
                                     buf, len(buf), C.byref(need))
        raise_for(rc, buf.value.decode(errors="replace"))
        return json.loads(buf.value.decode())


class PinnedWords:
    """A page-locked uint32 host array (kw_host_alloc) for verdict buffers a caller keeps: the bulk
    path reads verdicts back into it by direct DMA. `.array` is the numpy view.

    The allocation lives exactly as long as the ctypes buffer the view wraps (a weakref.finalize on
    it calls kw_host_free): any view or slice of `.array` keeps it alive, whether or not this
    wrapper still exists. close() only drops the wrapper's own reference."""

    def __init__(self, count, device=0):
        import numpy as np
        import weakref
        L = N.lib()
        p = C.c_void_p()
        raise_for(L.kw_host_alloc(device, max(count, 1) * 4, C.byref(p)), "kw_host_alloc failed")
        buf = (C.c_uint32 * max(count, 1)).from_address(p.value)
        self._free = weakref.finalize(buf, L.kw_host_free, C.c_void_p(p.value))
        self.array = np.frombuffer(buf, dtype=np.uint32, count=count)

    @property
    def alive(self):
        """True while the page-locked allocation exists (some view still references it)."""
        return self._free.alive

    def close(self):
        self.array = None


class Batch:
    """A micro-batch of requests in SoA form (kw_batch)."""

    def __init__(self, handle, keepalive=None):
        self._h = handle
        self._L = N.lib()
        self._keep = keepalive
        self.device = -1

    @classmethod
    def from_json(cls, documents, raw=False):
        L = N.lib()
        docs = [d.encode() if isinstance(d, str) else (json.dumps(d).encode() if isinstance(d, (dict, list)) else d)
                for d in documents]
        n = len(docs)
        arr = (C.c_char_p * max(n, 1))(*docs)
        lens = (C.c_size_t * max(n, 1))(*[len(d) for d in docs])
        h = C.c_void_p()
        bad = C.c_int64(-1)
        err = C.create_string_buffer(2048)
        rc = L.kw_batch_from_json(arr, lens, n, N.KW_DOC_RAW_REVIEW if raw else N.KW_DOC_ADMISSION_REVIEW,
                                  C.byref(h), C.byref(bad), err, len(err))
        if rc == N.KW_E_PAYLOAD:
            e = PayloadError(err.value.decode(errors="replace"))
            e.row = bad.value
            raise e
        raise_for(rc, err.value.decode(errors="replace"))
        return cls(h)

    @classmethod
    def from_soa(cls, soa, keepalive=None):
        L = N.lib()
        h = C.c_void_p()
        rc = L.kw_batch_from_soa(C.byref(soa), C.byref(h))
        raise_for(rc, "kw_batch_from_soa: inconsistent columns")
        return cls(h, keepalive)

    def view(self):
        s = KwSoa()
        raise_for(self._L.kw_batch_view(self._h, C.byref(s)), "view")
        s._owner = self  # the view points into this batch's columns
        return s

    @property
    def n(self):
        return self.view().n_requests

    def to_device(self, device=0):
        raise_for(self._L.kw_batch_to_device(self._h, device), f"kw_batch_to_device({device}) failed")
        self.device = device
        return self

    def validate(self, env, policies, origin=VALIDATE, stream=None):
        """All pairs rows x policies on the GPU; returns nothing (verdicts stay in HBM). stream: a
        hipStream_t (int) of the batch's device to run on, None = the batch's own stream."""
        arr = env._array(policies)
        rc = self._L.kw_validate_batch(env._h, self._h, arr, len(policies), origin,
                                       C.c_void_p(stream) if stream else None)
        raise_for(rc, "kw_validate_batch failed")
        self._npol = len(policies)

    def validate_rows(self, env, row_policy, origin=VALIDATE):
        arr = (C.c_int32 * len(row_policy))(*[env._idx(p) for p in row_policy])
        rc = self._L.kw_validate_rows(env._h, self._h, arr, origin, None)
        raise_for(rc, "kw_validate_rows failed")
        self._npol = 1

    def verdicts(self, count=None, out=None):
        """The last pass's verdict words (kw_batch_verdicts); `out`: a reused uint32 array to fill."""
        import numpy as np
        if count is None:
            count = self.n * self._npol if out is None else out.size
        if out is None:
            out = np.zeros(count, dtype=np.uint32)
        elif out.dtype != np.uint32 or not out.flags.c_contiguous or out.size < count:
            raise ValueError("out must be a contiguous uint32 array of at least count words")
        rc = self._L.kw_batch_verdicts(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), count)
        raise_for(rc, "kw_batch_verdicts failed")
        return out

    def pin_host(self, device=0):
        """Page-lock the batch's large host columns in place (kw_batch_pin_host): later bulk passes
        (validate_host) DMA them without the staging copy."""
        raise_for(self._L.kw_batch_pin_host(self._h, device), "kw_batch_pin_host failed")
        return self

    def validate_host(self, env, policies, out=None, origin=VALIDATE, device=0, chunk_rows=0):
        """Bulk host -> host pass (kw_validate_host): upload, evaluate and read back in overlapped row
        chunks; returns the [row][npol] verdict words in `out` (a reused uint32 array, pinned ones from
        PinnedWords read back by direct DMA)."""
        import numpy as np
        npol = len(policies)
        count = self.n * npol
        if out is None:
            out = np.empty(count, dtype=np.uint32)
        elif out.dtype != np.uint32 or not out.flags.c_contiguous or out.size < count:
            raise ValueError("out must be a contiguous uint32 array of at least rows x policies words")
        arr = (C.c_int32 * npol)(*[env._idx(p) for p in policies])
        rc = self._L.kw_validate_host(env._h, self._h, arr, npol, origin, device,
                                      out.ctypes.data_as(C.POINTER(C.c_uint32)), count, chunk_rows)
        raise_for(rc, "kw_validate_host failed")
        self.device = device
        self._npol = npol
        return out[:count]

    def debug_plan(self, env, policies, origin=VALIDATE):
        """Diagnostic (kw_debug_plan): the tile kernel's plan for an all-pairs pass, on the host."""
        arr = env._array(policies)
        out = (C.c_uint32 * 16)()
        raise_for(self._L.kw_debug_plan(env._h, self._h, arr, len(policies), origin, out, 16), "kw_debug_plan failed")
        keys = ("lds_bytes", "launches", "chunks", "lds_tables", "rows", "cmax", "kmax", "lmax", "regions", "split",
                "grid", "heavy_lds_bytes", "heavy_rows", "heavy_cmax", "heavy_grid", "scan_regions")
        return dict(zip(keys, out[:16]))

    def debug_reorder(self):
        """Diagnostic (kw_debug_reorder): the device-row order kw_batch_to_device gives this batch,
        as (batch in that order, perm, light-region rows); perm[d] is the batch row at device row d."""
        import numpy as np
        perm = np.zeros(max(self.n, 1), dtype=np.uint64)
        split, h = C.c_uint64(), C.c_void_p()
        rc = self._L.kw_debug_reorder(self._h, perm.ctypes.data_as(C.POINTER(C.c_uint64)), len(perm), C.byref(split),
                                      C.byref(h))
        raise_for(rc, "kw_debug_reorder failed")
        return Batch(h.value), perm[:self.n], split.value

    def wide_arg(self, row, policy):
        """Full argument of a verdict word whose ARG is KW_ARG_WIDE (kw_batch_wide_arg), or None."""
        v = C.c_uint64()
        rc = self._L.kw_batch_wide_arg(self._h, row, policy, C.byref(v))
        return v.value if rc == N.KW_OK else None

    def group_causes(self, row, policy, verdict):
        """Member slots (settings order) of a group rejection's causes (kw_batch_group_causes): from
        the word's ARG or the pass's side data, any number of members."""
        need = C.c_size_t()
        words = (C.c_uint64 * 1)()
        rc = self._L.kw_batch_group_causes(self._h, row, policy, int(verdict), words, 1, C.byref(need))
        if rc == N.KW_E_NOSPACE:
            words = (C.c_uint64 * need.value)()
            rc = self._L.kw_batch_group_causes(self._h, row, policy, int(verdict), words, need.value, C.byref(need))
        raise_for(rc, "kw_batch_group_causes")
        return [64 * k + b for k in range(need.value) for b in range(64) if (words[k] >> b) & 1]

    def debug_host_walk(self, env, policies, origin=VALIDATE):
        """Diagnostic (tests only): the device kernel's slot compiler + entity walks run on the host
        (kw_debug_host_walk). Never part of the validate path."""
        import numpy as np
        arr = env._array(policies)
        out = np.zeros(self.n * len(policies), dtype=np.uint32)
        rc = self._L.kw_debug_host_walk(env._h, self._h, arr, len(policies), origin,
                                        out.ctypes.data_as(C.POINTER(C.c_uint32)))
        raise_for(rc, "kw_debug_host_walk failed")
        return out

    def timed(self, env, policies, origin=VALIDATE, warmup=3, reps=10):
        arr = env._array(policies)
        t = KwTiming()
        rc = self._L.kw_validate_timed(env._h, self._h, arr, len(policies), origin, warmup, reps, C.byref(t))
        raise_for(rc, "kw_validate_timed failed")
        self._npol = len(policies)
        return t

    def format_response(self, env, row, policy, verdict, member_verdicts=None, doc=None, raw=False):
        """AdmissionResponse of (row, policy, verdict); `doc` (the row's original JSON) is needed
        for an accepted mutation, whose response carries the JSONPatch."""
        mv = None
        if member_verdicts is not None:
            mv = (C.c_uint32 * len(member_verdicts))(*[int(x) for x in member_verdicts])
        need = C.c_size_t()
        d = None if doc is None else (doc.encode() if isinstance(doc, str) else doc)

        def call(buf):
            if d is not None:
                return self._L.kw_format_response_doc(env._h, self._h, row, env._idx(policy), int(verdict), mv, d, len(d),
                                                      N.KW_DOC_RAW_REVIEW if raw else N.KW_DOC_ADMISSION_REVIEW, buf,
                                                      len(buf), C.byref(need))
            return self._L.kw_format_response(env._h, self._h, row, env._idx(policy), int(verdict), mv, buf, len(buf),
                                              C.byref(need))
        buf = C.create_string_buffer(1 << 15)
        rc = call(buf)
        if rc == N.KW_E_NOSPACE:  # a long response (a big JSONPatch): the size it needs
            buf = C.create_string_buffer(need.value + 1)
            rc = call(buf)
        raise_for(rc, buf.value.decode(errors="replace"))
        return json.loads(buf.value.decode())

    def close(self):
        if getattr(self, "_h", None):
            self._L.kw_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Metrics:
    """kubewarden_policy_evaluations_total and kubewarden_policy_evaluation_latency_milliseconds
    (src/metrics.rs:49-140), aggregated per validate pass from the verdict words (kw_metrics_*)."""

    def __init__(self):
        self._L = N.lib()
        self._h = self._L.kw_metrics_create()
        if not self._h:
            raise EngineError("kw_metrics_create failed")

    def record(self, env, batch, rows, policies, verdicts, latency_ms, origin=VALIDATE):
        n = len(rows)
        if not (len(policies) == len(verdicts) == len(latency_ms) == n):
            raise ValueError("rows, policies, verdicts and latency_ms must have the same length")
        r = (C.c_uint64 * max(n, 1))(*[int(x) for x in rows])
        p = (C.c_int32 * max(n, 1))(*[env._idx(x) if isinstance(x, str) else int(x) for x in policies])
        v = (C.c_uint32 * max(n, 1))(*[int(x) for x in verdicts])
        lat = (C.c_uint64 * max(n, 1))(*[int(x) for x in latency_ms])
        raise_for(self._L.kw_metrics_record(self._h, env._h, batch._h, r, p, v, lat, n, origin), "kw_metrics_record")

    def render(self):
        need = C.c_size_t(0)
        self._L.kw_metrics_render(self._h, None, 0, C.byref(need))
        buf = C.create_string_buffer(need.value + 1)
        raise_for(self._L.kw_metrics_render(self._h, buf, len(buf), C.byref(need)), "kw_metrics_render")
        return buf.value.decode()

    def samples(self):
        """{(metric name, frozenset of (label, value)): value} parsed from render()."""
        out = {}
        for line in self.render().splitlines():
            if not line or line.startswith("#"):
                continue
            head, val = line.rsplit(" ", 1)
            name, _, labels = head.partition("{")
            kv = []
            for part in _split_labels(labels.rstrip("}")):
                k, _, v = part.partition("=")
                kv.append((k, v[1:-1].replace('\\"', '"').replace("\\n", "\n").replace("\\\\", "\\")))
            out[(name, frozenset(kv))] = int(val)
        return out

    def reset(self):
        self._L.kw_metrics_reset(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.kw_metrics_destroy(self._h)
            self._h = None


def _split_labels(s):
    parts, cur, q, esc = [], "", False, False
    for ch in s:
        if esc:
            cur += ch
            esc = False
        elif ch == "\\":
            cur += ch
            esc = True
        elif ch == '"':
            cur += ch
            q = not q
        elif ch == "," and not q:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        parts.append(cur)
    return parts


def service_constraints(allowed, has_patch, has_status, mode, allowed_to_mutate):
    """validation_response_with_constraints (service.rs:160-208) on flags."""
    out = C.c_uint32()
    flags = (1 if allowed else 0) | (2 if has_patch else 0) | (4 if has_status else 0)
    fst = N.lib().kw_service_constraints(flags, mode, 1 if allowed_to_mutate else 0, C.byref(out))
    return fst, bool(out.value & 1), bool(out.value & 2), bool(out.value & 4)


def yaml_to_json(text):
    """The native host's YAML reader (kw_yaml_to_json): the JSON value of a YAML document."""
    b = text.encode() if isinstance(text, str) else text
    need = C.c_size_t()
    L = N.lib()
    L.kw_yaml_to_json(b, len(b), None, 0, C.byref(need))
    buf = C.create_string_buffer(need.value + 1)
    rc = L.kw_yaml_to_json(b, len(b), buf, len(buf), C.byref(need))
    if rc != N.KW_OK:
        raise ValueError(buf.value.decode(errors="replace"))
    return json.loads(buf.value.decode())


def pattern_match(kind, pattern, s):
    b = s.encode() if isinstance(s, str) else s
    return N.lib().kw_pattern_match(kind, pattern.encode(), b, len(b))


def pattern_match_many(kind, pattern, subjects):
    """kw_pattern_match_many: one compilation, a list of 1/0 per subject; None on a syntax error."""
    bs = [x.encode() if isinstance(x, str) else bytes(x) for x in subjects]
    n = len(bs)
    arr = (C.c_char_p * max(n, 1))(*bs)
    lens = (C.c_size_t * max(n, 1))(*[len(x) for x in bs])
    out = (C.c_int32 * max(n, 1))()
    if N.lib().kw_pattern_match_many(kind, pattern.encode(), arr, lens, n, out) != 0:
        return None
    return [int(out[k]) for k in range(n)]


def decode(v):
    """Verdict word -> dict (include/kwgpu.h layout)."""
    v = int(v)
    return {
        "allowed": bool(v & N.KW_V_ALLOWED), "mutated": bool(v & N.KW_V_MUTATED),
        "final_allowed": bool(v & N.KW_F_ALLOWED), "status": (v & N.KW_F_STATUS_MASK) >> N.KW_F_STATUS_SHIFT,
        "bypass": bool(v & N.KW_BYPASS), "patch": bool(v & N.KW_F_PATCH),
        "reason": N.REASONS.get((v >> 8) & 0xFF, (v >> 8) & 0xFF), "arg": v >> 16,
    }


class SynthBatch:
    """libkwsynth workload; .soa() is a kw_soa view valid while this object lives."""

    def __init__(self, config, n, seed, row0=0):
        self._S = N.synth()
        self._h = self._S.kws_generate(config, n, seed, row0)
        self.n = n

    def soa(self):
        s = KwSoa()
        self._S.kws_view(self._h, C.byref(s))
        s._owner = self  # the view points into this generator's columns
        return s

    def json(self, row):
        need = C.c_size_t()
        self._S.kws_json(self._h, row, None, 0, C.byref(need))
        buf = C.create_string_buffer(need.value)
        self._S.kws_json(self._h, row, buf, len(buf), C.byref(need))
        return buf.value.decode()

    def batch(self):
        return Batch.from_soa(self.soa(), keepalive=self)

    def __del__(self):
        try:
            self._S.kws_free(self._h)
        except Exception:
            pass
