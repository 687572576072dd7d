/*
 * kwgpu.h — C ABI of the MI355X batched admission-evaluation engine (libkwgpu.so).
 *
 * This is the drop-in boundary for the Kubewarden policy-server hot path
 *   POST /validate|/audit|/validate_raw/{policy_id}
 *     -> service::evaluate                      (src/api/service.rs:30-152)
 *     -> EvaluationEnvironment::validate        (src/evaluation/evaluation_environment.rs:546-556)
 * for the declarative policy class (namespace allow-list, trusted-repos, psp-capabilities,
 * psp-apparmor, safe-labels, pod-privileged, and policy groups over them).
 *
 * Every entry point names the reference interface it replaces. Plain pointers and sizes only:
 * no torch / HIP types appear in a signature ("stream" is an opaque hipStream_t or NULL).
 * All functions are thread-safe on a built (immutable) kw_env, like the reference's
 * Arc<EvaluationEnvironment> (src/lib.rs:194-197).
 */
#ifndef KWGPU_H
#define KWGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------------
 * Status codes. The first six mirror EvaluationError (src/evaluation/errors.rs:5-24) one to one;
 * the HTTP mapping of handle_evaluation_error (src/api/handlers.rs:321-342) is:
 * KW_E_NOT_FOUND -> 404 {"message":"unknown policy: <id>"}, every other error -> 500
 * {"message":"Something went wrong"}. KW_E_PAYLOAD is the 422 of JsonExtractor (handlers.rs:29-39).
 * ------------------------------------------------------------------------------------------- */
enum {
  KW_OK = 0,
  KW_E_INVALID_ID = 1,      /* EvaluationError::InvalidPolicyId        "Not a valid Policy ID: {0}" */
  KW_E_INIT = 2,            /* EvaluationError::PolicyInitialization   "{0}"                        */
  KW_E_NOT_FOUND = 3,       /* EvaluationError::PolicyNotFound         "unknown policy: {0}"        */
  KW_E_BOOTSTRAP = 4,       /* EvaluationError::BootstrapFailure       "bootstrap failure: {0}"     */
  KW_E_ENGINE = 5,          /* EvaluationError::WebAssemblyError slot: device/engine failure     */
  KW_E_GROUP_REHYDRATE = 6, /* EvaluationError::CannotRehydratePolicyGroup                        */
  KW_E_ARG = 16,            /* bad argument to this ABI                                           */
  KW_E_PAYLOAD = 17,        /* request JSON does not deserialize (HTTP 422)                       */
  KW_E_DEVICE = 18,         /* HIP runtime error                                                  */
  KW_E_NOSPACE = 19         /* caller buffer too small; *need holds the size                     */
};

/* PolicyMode (src/config.rs:287-294) */
enum { KW_MODE_PROTECT = 0, KW_MODE_MONITOR = 1 };
/* RequestOrigin (src/api/service.rs:16-19) */
enum { KW_ORIGIN_VALIDATE = 0, KW_ORIGIN_AUDIT = 1 };
/* ValidateRequest kind: AdmissionRequest vs Raw (service.rs:40, :134) */
enum { KW_DOC_ADMISSION_REVIEW = 0, KW_DOC_RAW_REVIEW = 1 };

/* ---------------------------------------------------------------------------------------------
 * Columnar (SoA) request batch. One row per ValidateRequest. Every string column is an offset
 * array (n+1 entries, u32) plus a byte pool; string i of a column belongs to entity i of that
 * column's table. Byte pools are padded to 16 B so device loads may over-read within the pad.
 * ------------------------------------------------------------------------------------------- */
typedef struct kw_strcol {
  const uint32_t *off;  /* n+1 offsets into bytes */
  const uint8_t *bytes; /* pool */
  uint64_t n;           /* number of strings */
} kw_strcol;

/* request flags */
enum {
  KW_REQ_RAW = 1u << 0,           /* ValidateRequest::Raw: namespace bypass is skipped (service.rs:40) */
  KW_REQ_HAS_NAMESPACE = 1u << 1, /* AdmissionRequest.namespace is Some */
  KW_REQ_HAS_PODSPEC = 1u << 2,   /* object carries a PodSpec (Pod or a workload template) */
  KW_REQ_HAS_OBJECT = 1u << 3     /* object is present and non-null */
};
/* container flags (containers, initContainers, ephemeralContainers, in that order) */
enum {
  KW_CTR_PRIVILEGED = 1u << 0,  /* securityContext.privileged == true */
  KW_CTR_INIT = 1u << 1,
  KW_CTR_EPHEMERAL = 1u << 2,
  KW_CTR_HAS_IMAGE = 1u << 3,
  KW_CTR_HAS_APPARMOR = 1u << 4 /* container.apparmor.security.beta.kubernetes.io/<name> annotation */
};

typedef struct kw_soa {
  uint64_t n_requests;
  /* per request */
  const uint8_t *req_flags; /* KW_REQ_* */
  const uint32_t *ctr_off;  /* n_requests+1: container range of each request */
  const uint32_t *lbl_off;  /* n_requests+1: metadata.labels range of each request */
  kw_strcol uid;            /* request.uid (host only, echoed in the response: service.rs:61,87) */
  kw_strcol ns;             /* request.namespace ("" when absent) */
  kw_strcol op;             /* request.operation */
  kw_strcol kind;           /* request.kind.kind */
  /* per container */
  const uint8_t *ctr_flags;   /* KW_CTR_* */
  const uint32_t *capadd_off; /* n_containers+1: securityContext.capabilities.add range */
  const uint32_t *capdrop_off;/* n_containers+1: securityContext.capabilities.drop range */
  kw_strcol ctr_name;
  kw_strcol ctr_image;
  kw_strcol ctr_apparmor; /* AppArmor profile from the pod annotation ("" when absent) */
  /* per capability entry */
  kw_strcol cap_add;
  kw_strcol cap_drop;
  /* per label */
  kw_strcol lbl_key;
  kw_strcol lbl_val;
} kw_soa;

/* ---------------------------------------------------------------------------------------------
 * Verdict word: one u32 per (row, policy) pair, written by the device.
 *   bit 0      V_ALLOWED   vanilla AdmissionResponse.allowed (the policy's own answer)
 *   bit 1      V_MUTATED   vanilla response carries a patch
 *   bit 2      F_ALLOWED   allowed after service::evaluate (bypass, init error, constraints)
 *   bits 3-4   F_STATUS    0: status None, 1: vanilla status, 2: mutation refused
 *                          (service.rs:168-180), 3: PolicyInitialization reject 500 (service.rs:78-91)
 *   bit 5      BYPASS      always-accept namespace (service.rs:40-71)
 *   bit 6      F_PATCH     the final response carries the vanilla patch (Audit, or Protect with
 *                          allowedToMutate)
 *   bits 8-15  REASON      kw_reason (0 = no violation)
 *   bits 16-31 ARG         reason argument: an entity index within the request, a settings index,
 *                          or a group's cause mask; KW_ARG_WIDE (0xffff) when the full value does
 *                          not fit (an index >= 65535, the causes of a group with more than 15
 *                          members): kw_batch_wide_arg returns it after kw_batch_verdicts
 * ------------------------------------------------------------------------------------------- */
#define KW_V_ALLOWED 0x1u
#define KW_V_MUTATED 0x2u
#define KW_F_ALLOWED 0x4u
#define KW_F_STATUS_SHIFT 3
#define KW_F_STATUS_MASK 0x18u
#define KW_BYPASS 0x20u
#define KW_F_PATCH 0x40u
#define KW_REASON(v) (((v) >> 8) & 0xffu)
#define KW_ARG(v) ((v) >> 16)
#define KW_ARG_WIDE 0xffffu
enum { KW_FST_NONE = 0, KW_FST_VANILLA = 1, KW_FST_MUTATION_REFUSED = 2, KW_FST_INIT_ERROR = 3 };

/* reason codes (message templates: DESIGN.md §Policy families) */
enum {
  KW_R_NONE = 0,
  KW_R_PRIVILEGED = 1,        /* arg: container index within the request */
  KW_R_NAMESPACE = 2,         /* namespace not the valid one */
  KW_R_REG_NOT_ALLOWED = 3,   /* arg: container index */
  KW_R_REG_REJECTED = 4,
  KW_R_TAG_REJECTED = 5,
  KW_R_IMG_NOT_ALLOWED = 6,
  KW_R_IMG_REJECTED = 7,
  KW_R_CAP_NOT_ALLOWED = 8,   /* arg: index in the request's capabilities.add lists, flattened in
                                 container order (the container is the one whose list holds it) */
  KW_R_APPARMOR = 9,          /* arg: container index */
  KW_R_LABEL_DENIED = 10,     /* arg: label index */
  KW_R_LABEL_CONSTRAINT = 11, /* arg: label index (the constraint is the policy's on that key) */
  KW_R_LABEL_MANDATORY = 12,  /* arg: index of the missing key in settings order */
  KW_R_GROUP = 13,            /* arg: cause mask over group members (settings order) */
  KW_R_GROUP_EXPR = 14,       /* group expression does not evaluate to a bool: reject 500 */
  KW_R_INIT_ERROR = 15
};

/* ---------------------------------------------------------------------------------------------
 * EvaluationEnvironment (src/evaluation/evaluation_environment.rs:86-127)
 * ------------------------------------------------------------------------------------------- */
typedef struct kw_env kw_env;

typedef struct kw_env_options {
  int continue_on_errors;              /* EvaluationEnvironmentBuilder::with_continue_on_errors :166 */
  const char *always_accept_namespace; /* ::with_always_accept_admission_reviews_on_namespace :172; NULL = None */
  int device;                          /* HIP device ordinal for the compiled tables; -1 = host only */
} kw_env_options;

/* EvaluationEnvironmentBuilder::build (evaluation_environment.rs:189-194, 198-332) plus the
 * policies.yml schema checks (src/config.rs:237-258, 287-453). `policies_json` is the policies file
 * as JSON (the reference converts YAML settings to JSON itself: config.rs:419-443). Compiles every
 * policy's settings into DFA/bitmask tables. On error returns the EvaluationError code and writes
 * its Display string into err. */
int kw_env_build(const char *policies_json, size_t len, const kw_env_options *opts, kw_env **out,
                 char *err, size_t errlen);
/* The same from the policies.yml text itself (read_policies_file + convert_yaml_map_to_json,
 * src/config.rs:419-453): YAML is converted to JSON, then built as above. A YAML error is a
 * KW_E_BOOTSTRAP. kw_yaml_to_json exposes the conversion (KW_E_PAYLOAD + message on error). */
int kw_env_build_yaml(const char *policies_yaml, size_t len, const kw_env_options *opts, kw_env **out,
                      char *err, size_t errlen);
int kw_yaml_to_json(const char *yaml, size_t len, char *buf, size_t cap, size_t *need);
/* Compiled-table blob (what rank 0 broadcasts over RCCL to the other GPUs). */
int kw_env_serialize(const kw_env *env, void *buf, size_t cap, size_t *need);
int kw_env_deserialize(const void *blob, size_t len, int device, kw_env **out, char *err, size_t errlen);
void kw_env_destroy(kw_env *env);

/* PolicyID::from_str (src/evaluation/policy_id.rs:29-47) + map lookup. Returns KW_OK and the
 * policy index, KW_E_INVALID_ID, or KW_E_NOT_FOUND. */
int kw_env_lookup(const kw_env *env, const char *policy_id, size_t len, int32_t *idx);
int kw_env_policy_count(const kw_env *env);
int kw_env_policy_id(const kw_env *env, int32_t idx, char *buf, size_t cap); /* PolicyID Display */
int kw_env_is_group(const kw_env *env, int32_t idx);
/* get_policy_mode / get_policy_allowed_to_mutate (evaluation_environment.rs:445-458) */
int kw_env_get_policy_mode(const kw_env *env, int32_t idx, int *mode);
int kw_env_get_policy_allowed_to_mutate(const kw_env *env, int32_t idx, int *allowed);
/* should_always_accept_requests_made_inside_of_namespace (evaluation_environment.rs:373-378) */
int kw_env_should_always_accept_requests_made_inside_of_namespace(const kw_env *env, const char *ns,
                                                                   size_t len);
/* policy_initialization_errors lookup (evaluation_environment.rs:569-571): 1 + message if set */
int kw_env_policy_initialization_error(const kw_env *env, int32_t idx, char *buf, size_t cap);
/* EvaluationEnvironment::validate_settings (evaluation_environment.rs:472-510): KW_OK, or
 * KW_E_INIT with the message (groups: expression validity, :496-506). */
int kw_env_validate_settings(const kw_env *env, int32_t idx, char *buf, size_t cap);
/* Diagnostic: does `s` match pattern `pat` (kind 0 literal, 1 glob, 2 regex) under the engine's
 * compiled-automaton semantics? 1/0, or -1 on a pattern syntax error. */
int kw_pattern_match(int kind, const char *pat, const char *s, size_t len);
/* The same for n subjects with one compilation: out[i] = 1/0; returns KW_OK, or -1 on a syntax
 * error. A pattern whose DFA exceeds the state budget runs as its NFA (kwdev.hpp DevNfa);
 * kind | KW_PATTERN_FORCE_NFA runs the NFA form whatever its DFA size (tests: DFA == NFA). */
#define KW_PATTERN_FORCE_NFA 0x100
int kw_pattern_match_many(int kind, const char *pat, const char *const *subjects, const size_t *lens, size_t n,
                          int32_t *out);
/* Diagnostics over the compiled classifiers (tests): the distinct patterns of request column `col`
 * (kwdev.hpp Col; kind 0 literal, 1 glob, 2 regex), and the ids of the patterns string `s` matches
 * through the blob's tables (the tables the kernels run). For COL_LV, `key` is the label key and
 * the result is restricted to the regexes constrained on it. kw_env_classify returns the number of
 * matched ids (writing at most `cap`), or -1. */
int kw_env_pattern_count(const kw_env *env, int col);
int kw_env_pattern(const kw_env *env, int col, int idx, int *kind, char *buf, size_t cap);
int kw_env_classify(const kw_env *env, int col, const char *key, size_t klen, const char *s, size_t len,
                    uint32_t *pats, int cap);

/* ---------------------------------------------------------------------------------------------
 * Request batches: the micro-batch handed over by the HTTP front (replaces the one
 * spawn_blocking task per request of acquire_semaphore_and_evaluate, handlers.rs:256-286).
 * ------------------------------------------------------------------------------------------- */
typedef struct kw_batch kw_batch;

/* Flatten n JSON documents (AdmissionReview {"request": AdmissionRequest} or RawReview
 * {"request": Value}) into SoA columns. A document that does not deserialize returns
 * KW_E_PAYLOAD with its row in *bad_row (the 422 of JsonExtractor, handlers.rs:29-39). */
int kw_batch_from_json(const char *const *docs, const size_t *lens, size_t n, int doc_kind,
                       kw_batch **out, int64_t *bad_row, char *err, size_t errlen);
/* Copy a caller-built SoA into a batch (the caller keeps ownership of its arrays). */
int kw_batch_from_soa(const kw_soa *soa, kw_batch **out);
/* Host view of the batch's columns (valid until kw_batch_destroy). */
int kw_batch_view(const kw_batch *b, kw_soa *view);
/* Upload the columns to HBM of `device` (synchronous; the bench times kernels with inputs resident).
 * Device memory and the pinned host staging come from per-device caching pools (returned when the
 * batch is destroyed), so a front that uploads thousands of micro-batches per second does not
 * allocate per batch. */
int kw_batch_to_device(kw_batch *b, int device);
/* The same, asynchronous on the caller's hipStream_t `stream` (which later passes of this batch use
 * by default); the upload completes in stream order. */
int kw_batch_to_device_async(kw_batch *b, int device, void *stream);
/* A non-blocking hipStream_t on `device` for callers without HIP headers (the HTTP front). */
int kw_stream_create(int device, void **stream);
void kw_stream_destroy(void *stream);
void kw_batch_destroy(kw_batch *b);

/* Diagnostic (test infrastructure, never called by kw_validate_*): evaluate the batch's rows
 * against the policy list on the HOST through the same slot compiler the device uses and the
 * sequential form of its first-violation walks (slots.hpp walk_*), with the column automata of the
 * blob. Lets the CPU test suite check the slot compiler against the oracle without a GPU.
 * out: [row][npol] verdict words. No reference counterpart (diagnostic only). */
int kw_debug_host_walk(const kw_env *env, const kw_batch *b, const int32_t *policies, uint32_t npol,
                       int origin, uint32_t *out);

/* Diagnostic (tests): plan an all-pairs pass over the batch's host columns without launching it.
 * out[0..8): LDS bytes per workgroup, launches, slot-plan chunks, classifiers staged in LDS (1) or
 * read from global memory (0), requests per tile, container / capability / label capacities (of the
 * first region). cap >= 16 adds out[8..16): regions (1, or 2 for a light / heavy split batch), the
 * light region's rows, the first region's grid, the heavy region's LDS bytes, requests per tile,
 * container capacity and grid, and a bit per region launched as the container wave-scan kernel. */
int kw_debug_plan(const kw_env *env, kw_batch *b, const int32_t *policies, uint32_t npol, int origin, uint32_t *out,
                  int cap);

/* Diagnostic (tests): the device-row order kw_batch_to_device gives this batch — the light / heavy
 * split (rows with more than 5 containers after the others when they are 1-50 % of
 * a batch of >= 2^18 rows and hold >= 30 % of its containers; KW_SPLIT=0 / 1 never / always) — as a
 * new host batch *out in that order. *split: the light region's rows (0: not split, *out in batch
 * order); perm[d] (cap >= rows) the batch row at device row d. */
int kw_debug_reorder(const kw_batch *b, uint64_t *perm, size_t cap, uint64_t *split, kw_batch **out);

/* ---------------------------------------------------------------------------------------------
 * The hot path: EvaluationEnvironment::validate + service::evaluate constraints, batched.
 * Evaluates every row against each of the npol policies (indices from kw_env_lookup) on the GPU;
 * verdict words are laid out row-major [row][npol]. Runs asynchronously on `stream` (a
 * hipStream_t of the batch's device; NULL = the batch's own stream) into the batch's device
 * verdict buffer; kw_batch_verdicts copies them to the host, synchronising with that stream. A pass
 * on another stream than the batch's previous pass first waits for the previous one.
 * ------------------------------------------------------------------------------------------- */
int kw_validate_batch(const kw_env *env, kw_batch *b, const int32_t *policies, uint32_t npol,
                      int origin, void *stream);
/* Micro-batch form: row r is evaluated against row_policy[r] only (one verdict per row), the
 * shape of many concurrent /validate/{policy_id} calls. */
int kw_validate_rows(const kw_env *env, kw_batch *b, const int32_t *row_policy, int origin,
                     void *stream);
int kw_batch_verdicts(kw_batch *b, uint32_t *host_out, size_t count);
/* Bulk form for callers that hand over host columns and want host verdicts (SURVEY §8(d) timing
 * mode 2): uploads the batch to `device`, evaluates every row against the npol policies and writes
 * the [row][npol] verdict words to host `out` (count = rows x npol). The batch is cut into chunks of
 * about chunk_rows rows (0: 262144) whose upload, evaluation and read-back overlap on three streams;
 * only the string columns the pass reads are uploaded (a later pass on the batch that needs others
 * returns KW_E_ARG until the batch is uploaded again). `out` may be pageable (read back through
 * pinned bounce blocks) or pinned (kw_host_alloc: direct DMA). Passes that need several launches,
 * overflow requests or wide side data run unchunked with the same result. Synchronous. Replaces,
 * for a bulk caller, the per-request loop of acquire_semaphore_and_evaluate (handlers.rs:256-286). */
int kw_validate_host(const kw_env *env, kw_batch *b, const int32_t *policies, uint32_t npol, int origin,
                     int device, uint32_t *out, size_t count, uint32_t chunk_rows);
/* Page-lock the batch's large host column arrays in place (hipHostRegister; undone by
 * kw_batch_destroy) so kw_validate_host sends them to the device by DMA from where they lie instead
 * of through the pinned staging its host workers fill. For a caller that runs several bulk passes
 * over one batch, or that builds batches once and keeps them; registering costs about as much as one
 * staging fill. Arrays under 64 KiB, and any the runtime declines, stay staged. No reference
 * counterpart (a host-memory option of the bulk entry point). */
int kw_batch_pin_host(kw_batch *b, int device);
/* Pinned (page-locked) host memory for verdict buffers a caller keeps (direct DMA), and its release. */
int kw_host_alloc(int device, size_t bytes, void **out);
void kw_host_free(void *p);
/* The full argument of a verdict word whose ARG is KW_ARG_WIDE, for (row, policy) of the last pass
 * whose verdicts were copied (kw_batch_verdicts). KW_E_NOT_FOUND when the pass recorded none. */
int kw_batch_wide_arg(const kw_batch *b, uint64_t row, int32_t policy, uint64_t *value);
/* The causes of a policy-group rejection (REASON KW_R_GROUP) of the last copied pass as a member
 * bitset (bit s: the group's member s, settings order, was called by the expression and rejected;
 * evaluation_environment.rs:979-1042): from the word's ARG, or the pass's side data for groups with
 * more than 15 members (any number of members: `words` holds ceil(members / 64) u64, `needed` gets
 * that count; KW_E_NOSPACE when nwords is smaller). Replaces the causes of
 * PolicyGroupEvaluator::validate's AdmissionResponse (upstream policy-evaluator). */
int kw_batch_group_causes(const kw_batch *b, uint64_t row, int32_t policy, uint32_t verdict, uint64_t *words,
                          size_t nwords, size_t *needed);

typedef struct kw_timing {
  double classify_ms;   /* 0: classification is fused into the evaluation kernel */
  double evaluate_ms;   /* avg device time of one whole validate pass (every launch of it) */
  double total_ms;      /* avg device time of one whole validate pass */
  double classify_bytes;/* 0 */
  double evaluate_bytes;/* algorithmic bytes per pass */
} kw_timing;
/* Time `reps` back-to-back validate passes with HIP events on the launch stream. */
int kw_validate_timed(const kw_env *env, kw_batch *b, const int32_t *policies, uint32_t npol,
                      int origin, int warmup, int reps, kw_timing *out);

/* ---------------------------------------------------------------------------------------------
 * Responses. Build the AdmissionResponse JSON of one (row, policy) from its verdict word, exactly
 * as service::evaluate would return it (uid echo, status message/code, group causes).
 * member_verdicts: verdict words of the group's members for this row (settings order) or NULL
 * for a non-group policy.
 * ------------------------------------------------------------------------------------------- */
int kw_format_response(const kw_env *env, const kw_batch *b, uint64_t row, int32_t policy,
                       uint32_t verdict, const uint32_t *member_verdicts, char *buf, size_t cap,
                       size_t *need);
/* The same with the row's original document (doc_kind KW_DOC_*), which an accepted mutation
 * (KW_F_PATCH) needs: the response then carries patchType "JSONPatch" and the base64 RFC 6902
 * patch that adds the psp-capabilities policy's missing required drops / default adds to every
 * container (the mutated_object of the guest, returned as a patch by policy-evaluator [upstream];
 * DESIGN.md §2). kw_format_response answers KW_E_ARG for such a verdict. */
int kw_format_response_doc(const kw_env *env, const kw_batch *b, uint64_t row, int32_t policy,
                           uint32_t verdict, const uint32_t *member_verdicts, const char *doc,
                           size_t doc_len, int doc_kind, char *buf, size_t cap, size_t *need);
/* Group member policy indices (settings order) of a group; returns the count. */
int kw_env_group_members(const kw_env *env, int32_t group, int32_t *out, int cap);

/* service::evaluate for one request, end to end (service.rs:30-152): PolicyID parse, namespace
 * bypass, validate on the device, constraints, response JSON. Returns KW_OK with the response,
 * or the EvaluationError code (with Display message in buf) that the handler maps to HTTP. */
int kw_evaluate(const kw_env *env, const char *policy_id, const char *doc, size_t doc_len,
                int doc_kind, int origin, char *buf, size_t cap, size_t *need);

/* validation_response_with_constraints (service.rs:160-208) on a vanilla response given as
 * flags, for the reference's own truth-table tests. in/out flags: bit0 allowed, bit1 has patch,
 * bit2 has status. Returns the F_STATUS kind of the result. */
int kw_service_constraints(uint32_t vanilla_flags, int mode, int allowed_to_mutate,
                           uint32_t *out_flags);

/* ---------------------------------------------------------------------------------------------
 * Metrics (src/metrics.rs:49-140, src/metrics/policy_evaluations_{total,latency}.rs; recorded by
 * service::evaluate, src/api/service.rs:40-71, :78-84, :118-150). A kw_metrics aggregates the
 * counter kubewarden_policy_evaluations_total and the u64 histogram
 * kubewarden_policy_evaluation_latency_milliseconds with the reference's attribute sets:
 *   AdmissionRequest: policy_name, policy_mode, resource_kind (requestKind.kind),
 *     resource_request_operation, accepted, mutated, request_origin[, resource_namespace][, error_code]
 *   Raw: policy_name, policy_mode, accepted, mutated[, error_code]
 *   initialization error (counter only): policy_name, initialization_error
 * accepted / mutated / error_code are the vanilla response's (before constraints); a namespace
 * bypass counts as accepted, not mutated. Thread-safe; kept off the device path.
 * ------------------------------------------------------------------------------------------- */
typedef struct kw_metrics kw_metrics;
kw_metrics *kw_metrics_create(void);
void kw_metrics_destroy(kw_metrics *m);
/* Record n evaluated (row, policy) pairs of one validate pass: rows[i] of batch b against
 * policies[i], with their final verdict words and the latency from arrival to verdict in ms. Only
 * the policies the requests addressed are recorded (not a group's member rows). */
int kw_metrics_record(kw_metrics *m, const kw_env *env, const kw_batch *b, const uint64_t *rows,
                      const int32_t *policies, const uint32_t *verdicts, const uint64_t *latency_ms,
                      size_t n, int origin);
/* Prometheus text exposition (format 0.0.4) of everything recorded so far. */
int kw_metrics_render(const kw_metrics *m, char *buf, size_t cap, size_t *need);
void kw_metrics_reset(kw_metrics *m);

const char *kw_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KWGPU_H */
