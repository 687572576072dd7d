/*
 * kworacle.h — CPU restatement of the declarative-policy hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline — never as a product path. The product
 * (libkwgpu.so) has no link to it and fails loudly without its HIP kernels.
 *
 * What it restates (reference file:line):
 *   - EvaluationEnvironment::validate_policy dispatch (src/evaluation/evaluation_environment.rs:546-581)
 *   - the per-policy arithmetic of the declarative class, which upstream lives in Wasm modules that
 *     are NOT in /root/reference (policy-evaluator v0.24.0 @ f097b70a, Cargo.lock:4308-4347; OCI
 *     modules named in policies.yml.example:1-33). Parity for these families is UNPINNED: the
 *     semantics follow the spec in DESIGN.md §"Policy families", except pod-privileged whose
 *     message is pinned by tests/integration_test.rs:58-68.
 *   - service::evaluate namespace bypass + validation_response_with_constraints
 *     (src/api/service.rs:40-71, 78-91, 108-116, 160-208): pinned by service.rs:285-718.
 *   - PolicyGroupEvaluator short-circuit semantics [upstream, rhai 1.21.0] as exercised by
 *     evaluation_environment.rs:979-1042 and integration_test.rs:101-131, 204-251.
 * It consumes the kw_soa columns declared in include/kwgpu.h (the boundary's data format) and an
 * oracle-side policy description built by oracle/oracle.py from the parsed policies document.
 * Strings are matched with libc fnmatch(3) (globs) and the oracle's own regex matcher (kwregex.c) —
 * an implementation independent of the product's DFA compiler.
 */
#ifndef KWORACLE_H
#define KWORACLE_H
#include <stdint.h>
#include "../include/kwgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORC_F_PRIVILEGED = 1,
  ORC_F_NAMESPACE = 2,
  ORC_F_TRUSTED_REPOS = 3,
  ORC_F_CAPABILITIES = 4,
  ORC_F_APPARMOR = 5,
  ORC_F_LABELS = 6,
  ORC_F_GROUP = 7
};

/* group expression tree node (built by oracle.py's own parser of the rhai subset) */
enum { ORC_X_CONST = 0, ORC_X_CALL = 1, ORC_X_NOT = 2, ORC_X_AND = 3, ORC_X_OR = 4, ORC_X_EQ = 5, ORC_X_NE = 6 };
typedef struct orc_xnode {
  int32_t op;
  int32_t a; /* CONST: 0/1; CALL: member slot; NOT/AND/OR/EQ/NE: left child */
  int32_t b; /* AND/OR/EQ/NE: right child */
} orc_xnode;

typedef struct orc_policy {
  int32_t family;
  int32_t mode;              /* KW_MODE_* */
  int32_t allowed_to_mutate;
  int32_t init_error;        /* PolicyInitialization recorded under continue_on_errors */
  int32_t expr_error;        /* group: expression does not evaluate to a bool */
  int32_t flags;             /* bit0 skip_init_containers, bit1 skip_ephemeral_containers,
                                bit2 allowed_capabilities contains "*" */
  /* string lists (meaning per family):
     namespace:     l0 = [valid_namespace]
     trusted-repos: l0 reg allow, l1 reg reject, l2 tag reject, l3 image allow, l4 image reject (globs)
     capabilities:  l0 allowed, l1 required_drop, l2 default_add
     apparmor:      l0 allowed_profiles
     labels:        l0 denied, l1 mandatory, l2 constrained keys, l3 constrained regexes */
  int32_t n[5];
  const char *const *l[5];
  /* group */
  int32_t n_members;
  const int32_t *members;   /* policy indices, settings order */
  int32_t n_nodes;
  const orc_xnode *nodes;   /* root = nodes[n_nodes-1] */
  /* group scripts outside the bool-only subset (let / if / strings / integers, <= 16 members):
     oracle.py's own interpreter tabulated over every vector of member results, entry[mask] =
     bit 0 value, bit 1 evaluation error, bits 16.. the members called that rejected; every member
     is evaluated, the entry picks the outcome; NULL = evaluate `nodes` */
  const uint32_t *table;
} orc_policy;

typedef struct orc_env orc_env;
/* Compiles the regexes once; returns NULL and writes err on an invalid regex. */
orc_env *orc_env_new(const orc_policy *policies, int32_t npol, const char *always_accept_ns,
                     char *err, int errlen);
void orc_env_free(orc_env *e);

/* Verdict words (include/kwgpu.h layout) for rows [row0,row1) x policies, row-major. */
void orc_eval(const orc_env *e, const kw_soa *soa, const int32_t *policies, int32_t npol,
              int32_t origin, uint64_t row0, uint64_t row1, uint32_t *out);
/* Same, split over `threads` POSIX threads (the CPU baseline). */
void orc_eval_mt(const orc_env *e, const kw_soa *soa, const int32_t *policies, int32_t npol,
                 int32_t origin, uint64_t nrows, int threads, uint32_t *out);
/* Same, thread t pinned to CPU cpus[t] (cpus may be NULL). */
void orc_eval_mt_pinned(const orc_env *e, const kw_soa *soa, const int32_t *policies, int32_t npol, int32_t origin,
                        uint64_t nrows, int threads, const int32_t *cpus, uint32_t *out);

/* What one (row, policy) evaluation found, before any encoding into a verdict word: the response
   is derived from this and the document, never from the product's word (oracle.py response_doc).
   arg: the FULL argument (entity index within the request, settings index); causes: the group
   members rhai would have called that rejected, ascending member slots. */
#define ORC_MAX_MEMBERS 4096
typedef struct orc_detail {
  uint32_t word;      /* the verdict word (kwgpu.h layout, ARG saturated to KW_ARG_WIDE) */
  uint32_t reason;    /* KW_R_* of the vanilla response, 0 = accepted */
  uint64_t arg;       /* full argument of `reason` */
  uint32_t mutated;   /* the vanilla response carries a patch */
  uint32_t bypass;    /* namespace bypass (service.rs:40-71) */
  int32_t ncauses;
  int32_t causes[ORC_MAX_MEMBERS];
} orc_detail;
void orc_eval_detail(const orc_env *e, const kw_soa *soa, int32_t policy, int32_t origin, uint64_t row, orc_detail *out);

/* 1 if the regex compiles in the dialect of DESIGN.md §2 (kwregex.c). */
int orc_regex_ok(const char *pattern);

/* kwregex.c: the oracle's own matcher for that dialect (Rust `regex` syntax, Regex::is_match
   search semantics, a Pike VM over code points). NULL with a message on a syntax error. */
typedef struct orc_re orc_re;
orc_re *orc_re_compile(const char *pattern, char *err, int errlen);
int orc_re_search(const orc_re *re, const char *s, size_t n);
void orc_re_free(orc_re *re);
/* convenience for tests: 1 match, 0 no match, -1 the pattern does not compile */
int orc_re_match(const char *pattern, const char *s, size_t n);

/* kwregex.c: globs (fnmatch(3) flags 0 over code points), independent of the locale.
   orc_glob_ok: 1 if the glob is supported; orc_glob_match: 1 match, 0 no match, -1 unsupported. */
int orc_glob_ok(const char *pattern);
int orc_glob_match(const char *pattern, const char *s, size_t n);
/* compiled once (per environment): NULL when unsupported; run: 1 match, 0 no match */
typedef struct orc_glob orc_glob;
orc_glob *orc_glob_compile(const char *pattern);
int orc_glob_run(const orc_glob *g, const char *s, size_t n);
void orc_glob_free(orc_glob *g);

/* Image reference normalisation; writes NUL-terminated parts.
   Returns 1 if an effective tag exists. */
int orc_image_parts(const char *image, char *registry, char *tag, char *normalized, int cap);

#ifdef __cplusplus
}
#endif
#endif
