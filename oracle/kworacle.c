/*
 * kworacle.c — CPU restatement of the declarative-policy hot path. TEST INFRASTRUCTURE ONLY
 * (see kworacle.h for what is restated, from which reference file:line, and who may load it).
 * Parity status: service constraints / bypass / group short-circuit are pinned by the reference's
 * own tests (tests/golden/); the policy-family arithmetic is parity UNPINNED (upstream Wasm absent)
 * and follows DESIGN.md §"Policy families".
 */
#define _GNU_SOURCE
#include "kworacle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

struct orc_env {
  const orc_policy *pol;
  int32_t npol;
  char *always_ns; /* NULL = None */
  orc_re ***re;    /* per policy: compiled l3 regexes (labels) */
  orc_glob ***gl;  /* per policy: its five glob lists compiled, concatenated (trusted-repos) */
};

static char *dupz(const char *s) {
  size_t n = strlen(s);
  char *d = (char *)malloc(n + 1);
  memcpy(d, s, n + 1);
  return d;
}

orc_env *orc_env_new(const orc_policy *policies, int32_t npol, const char *always_ns, char *err,
                     int errlen) {
  orc_env *e = (orc_env *)calloc(1, sizeof(orc_env));
  e->pol = policies;
  e->npol = npol;
  e->always_ns = always_ns ? dupz(always_ns) : NULL;
  e->re = (orc_re ***)calloc((size_t)npol, sizeof(orc_re **));
  e->gl = (orc_glob ***)calloc((size_t)npol, sizeof(orc_glob **));
  for (int32_t p = 0; p < npol; ++p) {
    const orc_policy *P = &policies[p];
    if (P->family == ORC_F_TRUSTED_REPOS && !P->init_error) {
      const int32_t tot = P->n[0] + P->n[1] + P->n[2] + P->n[3] + P->n[4];
      e->gl[p] = (orc_glob **)calloc((size_t)tot + 1, sizeof(orc_glob *));
      int32_t at = 0;
      for (int k = 0; k < 5; ++k)
        for (int32_t i = 0; i < P->n[k]; ++i) e->gl[p][at++] = orc_glob_compile(P->l[k][i]);  /* NULL never matches */
    }
    if (P->family != ORC_F_LABELS || P->n[3] == 0 || P->init_error) continue;
    e->re[p] = (orc_re **)calloc((size_t)P->n[3], sizeof(orc_re *));
    for (int32_t i = 0; i < P->n[3]; ++i) {
      e->re[p][i] = orc_re_compile(P->l[3][i], err, errlen);
      if (!e->re[p][i]) {
        e->npol = p + 1;
        orc_env_free(e);
        return NULL;
      }
    }
  }
  return e;
}

void orc_env_free(orc_env *e) {
  if (!e) return;
  for (int32_t p = 0; p < e->npol; ++p) {
    if (e->gl[p]) {
      const orc_policy *P = &e->pol[p];
      const int32_t tot = P->n[0] + P->n[1] + P->n[2] + P->n[3] + P->n[4];
      for (int32_t i = 0; i < tot; ++i) orc_glob_free(e->gl[p][i]);
      free(e->gl[p]);
    }
    if (!e->re[p]) continue;
    for (int32_t i = 0; i < e->pol[p].n[3]; ++i) orc_re_free(e->re[p][i]);
    free(e->re[p]);
  }
  free(e->re);
  free(e->gl);
  free(e->always_ns);
  free(e);
}

int orc_regex_ok(const char *pattern) {
  orc_re *re = orc_re_compile(pattern, NULL, 0);
  orc_re_free(re);
  return re != NULL;
}

int orc_re_match(const char *pattern, const char *s, size_t n) {
  orc_re *re = orc_re_compile(pattern, NULL, 0);
  if (!re) return -1;
  int r = orc_re_search(re, s, n);
  orc_re_free(re);
  return r;
}

/* ------------------------------------------------------------------ string helpers */
typedef struct {
  const char *p;
  uint32_t n;
} sv;

static sv col(const kw_strcol *c, uint64_t i) {
  sv s;
  s.p = (const char *)c->bytes + c->off[i];
  s.n = c->off[i + 1] - c->off[i];
  return s;
}

/* NUL-terminated scratch copy (strings are short; long ones get a heap buffer) */
typedef struct {
  char small[512];
  char *big;
} zbuf;
static const char *z(zbuf *b, sv s) {
  char *d = b->small;
  if (s.n + 1 > sizeof(b->small)) {
    free(b->big);
    b->big = (char *)malloc(s.n + 1);
    d = b->big;
  }
  memcpy(d, s.p, s.n);
  d[s.n] = 0;
  return d;
}

static int sv_eq(sv s, const char *t) { return strlen(t) == s.n && memcmp(s.p, t, s.n) == 0; }

static int any_glob(orc_glob *const *g, int32_t n, const char *s) {
  const size_t len = strlen(s);
  for (int32_t i = 0; i < n; ++i)
    if (g[i] && orc_glob_run(g[i], s, len) == 1) return 1;
  return 0;
}
static int any_eq(const char *const *lst, int32_t n, sv s) {
  for (int32_t i = 0; i < n; ++i)
    if (sv_eq(s, lst[i])) return 1;
  return 0;
}

/* ------------------------------------------------------------------ image references */
/* DESIGN.md §trusted-repos "image reference normalisation":
   name@digest split at the first '@'; the first '/'-component is a registry iff it contains '.'
   or ':' or equals "localhost", else the registry is docker.io; the tag is what follows the last
   ':' of the remainder; docker.io single-component paths get "library/"; the effective tag is the
   explicit tag, else "latest" when there is no digest, else none. */
int orc_image_parts(const char *s, char *registry, char *tag, char *norm, int cap) {
  (void)cap;
  size_t n = strlen(s);
  const char *at = memchr(s, '@', n);
  size_t name_n = at ? (size_t)(at - s) : n;
  const char *slash = memchr(s, '/', name_n);
  size_t reg_b = 0, reg_n = 0, rest_b = 0;
  int explicit_reg = 0;
  if (slash) {
    size_t c0 = (size_t)(slash - s);
    int isreg = (memchr(s, '.', c0) != NULL) || (memchr(s, ':', c0) != NULL) ||
                (c0 == 9 && memcmp(s, "localhost", 9) == 0);
    if (isreg) {
      explicit_reg = 1;
      reg_b = 0;
      reg_n = c0;
      rest_b = c0 + 1;
    }
  }
  if (explicit_reg) {
    memcpy(registry, s + reg_b, reg_n);
    registry[reg_n] = 0;
  } else {
    strcpy(registry, "docker.io");
  }
  size_t rest_n = name_n - rest_b;
  const char *rest = s + rest_b;
  const char *colon = NULL;
  for (size_t i = rest_n; i > 0; --i)
    if (rest[i - 1] == ':') {
      colon = rest + i - 1;
      break;
    }
  size_t path_n = colon ? (size_t)(colon - rest) : rest_n;
  int has_tag = colon != NULL;
  int is_docker = strcmp(registry, "docker.io") == 0;
  int path_slash = memchr(rest, '/', path_n) != NULL;
  int eff_tag = 1;
  if (has_tag) {
    size_t tn = rest_n - path_n - 1;
    memcpy(tag, colon + 1, tn);
    tag[tn] = 0;
  } else if (!at) {
    strcpy(tag, "latest");
  } else {
    tag[0] = 0;
    eff_tag = 0;
  }
  char *w = norm;
  size_t rl = strlen(registry);
  memcpy(w, registry, rl);
  w += rl;
  *w++ = '/';
  if (is_docker && !path_slash) {
    memcpy(w, "library/", 8);
    w += 8;
  }
  memcpy(w, rest, path_n);
  w += path_n;
  if (eff_tag) {
    *w++ = ':';
    size_t tl = strlen(tag);
    memcpy(w, tag, tl);
    w += tl;
  }
  if (at) {
    size_t dn = n - name_n;
    memcpy(w, at, dn); /* '@' + digest */
    w += dn;
  }
  *w = 0;
  return eff_tag;
}

/* ------------------------------------------------------------------ families */
/* Full arguments: an entity index within the request (containers; capabilities.add entries
   flattened in container order; labels) or a settings index. The verdict word carries them in 16
   bits, KW_ARG_WIDE when they do not fit (include/kwgpu.h). */
typedef struct {
  uint32_t reason;
  uint64_t arg;
  uint32_t mutated;
} fam_out;

static int ctr_considered(const orc_policy *P, uint8_t f) {
  if ((P->flags & 1) && (f & KW_CTR_INIT)) return 0;
  if ((P->flags & 2) && (f & KW_CTR_EPHEMERAL)) return 0;
  return 1;
}

static fam_out fam_privileged(const orc_policy *P, const kw_soa *S, uint64_t r) {
  fam_out o = {0, 0, 0};
  if (!(S->req_flags[r] & KW_REQ_HAS_PODSPEC)) return o;
  for (uint32_t c = S->ctr_off[r]; c < S->ctr_off[r + 1]; ++c) {
    uint8_t f = S->ctr_flags[c];
    if (ctr_considered(P, f) && (f & KW_CTR_PRIVILEGED)) {
      o.reason = KW_R_PRIVILEGED;
      o.arg = c - S->ctr_off[r];
      return o;
    }
  }
  return o;
}

static fam_out fam_namespace(const orc_policy *P, const kw_soa *S, uint64_t r) {
  fam_out o = {0, 0, 0};
  sv ns = col(&S->ns, r);
  int ok = (S->req_flags[r] & KW_REQ_HAS_NAMESPACE) && P->n[0] > 0 && sv_eq(ns, P->l[0][0]);
  if (!ok) o.reason = KW_R_NAMESPACE;
  return o;
}

static fam_out fam_trusted(const orc_policy *P, orc_glob *const *G, const kw_soa *S, uint64_t r, zbuf *zb) {
  fam_out o = {0, 0, 0};
  if (!G) return o; /* (an init-error policy is answered before its family runs) */
  orc_glob *const *g[5];  /* the compiled lists l[0..4] */
  for (int k = 0, at = 0; k < 5; at += P->n[k], ++k) g[k] = G + at;
  if (!(S->req_flags[r] & KW_REQ_HAS_PODSPEC)) return o;
  char sreg[512], stag[512], snorm[1024];
  for (uint32_t c = S->ctr_off[r]; c < S->ctr_off[r + 1]; ++c) {
    uint8_t f = S->ctr_flags[c];
    if (!(f & KW_CTR_HAS_IMAGE)) continue;
    sv im = col(&S->ctr_image, c);
    char *reg = sreg, *tag = stag, *norm = snorm, *heap = NULL;
    if (im.n + 32 > sizeof(sreg)) { /* long references: scratch on the heap */
      heap = (char *)malloc(4 * (size_t)im.n + 128);
      reg = heap;
      tag = heap + im.n + 32;
      norm = heap + 2 * (size_t)im.n + 64;
    }
    int eff = orc_image_parts(z(zb, im), reg, tag, norm, 0);
    uint32_t why = 0;
    if (P->n[0] > 0 && !any_glob(g[0], P->n[0], reg))
      why = KW_R_REG_NOT_ALLOWED;
    else if (P->n[1] > 0 && any_glob(g[1], P->n[1], reg))
      why = KW_R_REG_REJECTED;
    else if (eff && P->n[2] > 0 && any_glob(g[2], P->n[2], tag))
      why = KW_R_TAG_REJECTED;
    else if (P->n[3] > 0 && !any_glob(g[3], P->n[3], norm))
      why = KW_R_IMG_NOT_ALLOWED;
    else if (P->n[4] > 0 && any_glob(g[4], P->n[4], norm))
      why = KW_R_IMG_REJECTED;
    free(heap);
    if (why) {
      o.reason = why;
      o.arg = c - S->ctr_off[r];
      return o;
    }
  }
  return o;
}

static fam_out fam_caps(const orc_policy *P, const kw_soa *S, uint64_t r) {
  fam_out o = {0, 0, 0};
  if (!(S->req_flags[r] & KW_REQ_HAS_PODSPEC)) return o;
  int allow_all = (P->flags & 4) != 0;
  /* validation: every added capability must be allowed (allowed_capabilities or
     default_add_capabilities), unless allowed_capabilities contains "*" */
  for (uint32_t c = S->ctr_off[r]; c < S->ctr_off[r + 1]; ++c) {
    if (allow_all) break;
    for (uint32_t k = S->capadd_off[c]; k < S->capadd_off[c + 1]; ++k) {
      sv cap = col(&S->cap_add, k);
      if (!any_eq(P->l[0], P->n[0], cap) && !any_eq(P->l[2], P->n[2], cap)) {
        o.reason = KW_R_CAP_NOT_ALLOWED;
        o.arg = k - S->capadd_off[S->ctr_off[r]];
        return o;
      }
    }
  }
  /* mutation: a container that does not drop a required capability (and does not drop ALL), or
     that neither adds nor drops a default capability, gets a patch */
  for (uint32_t c = S->ctr_off[r]; c < S->ctr_off[r + 1]; ++c) {
    int drop_all = 0;
    for (uint32_t k = S->capdrop_off[c]; k < S->capdrop_off[c + 1]; ++k)
      if (sv_eq(col(&S->cap_drop, k), "ALL")) drop_all = 1;
    for (int32_t i = 0; i < P->n[1] && !drop_all; ++i) {
      int dropped = 0;
      for (uint32_t k = S->capdrop_off[c]; k < S->capdrop_off[c + 1]; ++k)
        if (sv_eq(col(&S->cap_drop, k), P->l[1][i])) dropped = 1;
      if (!dropped) o.mutated = 1;
    }
    for (int32_t i = 0; i < P->n[2]; ++i) {
      int seen = 0;
      for (uint32_t k = S->capadd_off[c]; k < S->capadd_off[c + 1]; ++k)
        if (sv_eq(col(&S->cap_add, k), P->l[2][i])) seen = 1;
      for (uint32_t k = S->capdrop_off[c]; k < S->capdrop_off[c + 1]; ++k)
        if (sv_eq(col(&S->cap_drop, k), P->l[2][i])) seen = 1;
      if (!seen) o.mutated = 1;
    }
  }
  return o;
}

static fam_out fam_apparmor(const orc_policy *P, const kw_soa *S, uint64_t r) {
  fam_out o = {0, 0, 0};
  if (!(S->req_flags[r] & KW_REQ_HAS_PODSPEC)) return o;
  for (uint32_t c = S->ctr_off[r]; c < S->ctr_off[r + 1]; ++c) {
    if (!(S->ctr_flags[c] & KW_CTR_HAS_APPARMOR)) continue;
    if (!any_eq(P->l[0], P->n[0], col(&S->ctr_apparmor, c))) {
      o.reason = KW_R_APPARMOR;
      o.arg = c - S->ctr_off[r];
      return o;
    }
  }
  return o;
}

static fam_out fam_labels(const orc_env *e, int32_t p, const kw_soa *S, uint64_t r, zbuf *zb) {
  const orc_policy *P = &e->pol[p];
  fam_out o = {0, 0, 0};
  (void)zb;
  for (uint32_t l = S->lbl_off[r]; l < S->lbl_off[r + 1]; ++l) {
    sv key = col(&S->lbl_key, l);
    if (any_eq(P->l[0], P->n[0], key)) {
      o.reason = KW_R_LABEL_DENIED;
      o.arg = l - S->lbl_off[r];
      return o;
    }
    for (int32_t i = 0; i < P->n[2]; ++i) {
      if (!sv_eq(key, P->l[2][i])) continue;
      sv v = col(&S->lbl_val, l);
      if (!orc_re_search(e->re[p][i], v.p, v.n)) {
        o.reason = KW_R_LABEL_CONSTRAINT;
        o.arg = l - S->lbl_off[r];
        return o;
      }
    }
  }
  for (int32_t i = 0; i < P->n[1]; ++i) {
    int present = 0;
    for (uint32_t l = S->lbl_off[r]; l < S->lbl_off[r + 1]; ++l)
      if (sv_eq(col(&S->lbl_key, l), P->l[1][i])) present = 1;
    if (!present) {
      o.reason = KW_R_LABEL_MANDATORY;
      o.arg = (uint32_t)i;
      return o;
    }
  }
  return o;
}

static fam_out eval_family(const orc_env *e, int32_t p, const kw_soa *S, uint64_t r, zbuf *zb) {
  const orc_policy *P = &e->pol[p];
  fam_out none = {0, 0, 0};
  switch (P->family) {
  case ORC_F_PRIVILEGED: return fam_privileged(P, S, r);
  case ORC_F_NAMESPACE: return fam_namespace(P, S, r);
  case ORC_F_TRUSTED_REPOS: return fam_trusted(P, e->gl[p], S, r, zb);
  case ORC_F_CAPABILITIES: return fam_caps(P, S, r);
  case ORC_F_APPARMOR: return fam_apparmor(P, S, r);
  case ORC_F_LABELS: return fam_labels(e, p, S, r, zb);
  default: return none;
  }
}

/* ------------------------------------------------------------------ groups (short-circuit) */
typedef struct {
  const orc_env *e;
  const orc_policy *G;
  const kw_soa *S;
  uint64_t r;
  zbuf *zb;
  uint8_t done[ORC_MAX_MEMBERS], ok[ORC_MAX_MEMBERS];
} gctx;

/* member "returns true" iff allowed and not mutated (a patch inside a group is refused,
   integration_test.rs:247-250); evaluation is lazy, as rhai evaluates || and && */
static int gcall(gctx *g, int32_t slot) {
  if (!g->done[slot]) {
    g->done[slot] = 1;
    if (g->e->pol[g->G->members[slot]].init_error) {
      /* a member that failed to initialise never accepts (a cause when evaluated); the response
         layer answers such a group with PolicyNotFound for that member (oracle.py) */
      g->ok[slot] = 0;
    } else {
      fam_out fo = eval_family(g->e, g->G->members[slot], g->S, g->r, g->zb);
      g->ok[slot] = fo.reason == 0 && !fo.mutated;
    }
  }
  return g->ok[slot];
}
static int geval(gctx *g, int32_t n) {
  const orc_xnode *x = &g->G->nodes[n];
  switch (x->op) {
  case ORC_X_CONST: return x->a != 0;
  case ORC_X_CALL: return gcall(g, x->a);
  case ORC_X_NOT: return !geval(g, x->a);
  case ORC_X_AND: return geval(g, x->a) ? geval(g, x->b) : 0;
  case ORC_X_OR: return geval(g, x->a) ? 1 : geval(g, x->b);
  case ORC_X_EQ: { int l = geval(g, x->a); return l == geval(g, x->b); }
  case ORC_X_NE: { int l = geval(g, x->a); return l != geval(g, x->b); }
  }
  return 0;
}

/* ------------------------------------------------------------------ service::evaluate */
static void detail(const orc_env *e, int32_t p, const kw_soa *S, uint64_t r, int32_t origin, zbuf *zb, orc_detail *d) {
  const orc_policy *P = &e->pol[p];
  d->reason = 0;
  d->arg = 0;
  d->mutated = 0;
  d->bypass = 0;
  d->ncauses = 0;
  /* namespace bypass first (service.rs:40-71): AdmissionRequest only */
  if (e->always_ns && !(S->req_flags[r] & KW_REQ_RAW) && (S->req_flags[r] & KW_REQ_HAS_NAMESPACE) &&
      sv_eq(col(&S->ns, r), e->always_ns)) {
    d->bypass = 1;
    d->word = KW_V_ALLOWED | KW_F_ALLOWED | KW_BYPASS;
    return;
  }
  /* PolicyInitialization -> reject(uid, msg, 500), before any constraint (service.rs:78-91) */
  if (P->init_error) {
    d->reason = KW_R_INIT_ERROR;
    d->word = ((uint32_t)KW_FST_INIT_ERROR << KW_F_STATUS_SHIFT) | ((uint32_t)KW_R_INIT_ERROR << 8);
    return;
  }
  uint32_t arg16 = 0;
  if (P->family == ORC_F_GROUP) {
    if (P->expr_error) {
      d->reason = KW_R_GROUP_EXPR;
    } else if (P->table) {
      gctx g;
      g.e = e;
      g.G = P;
      g.S = S;
      g.r = r;
      g.zb = zb;
      memset(g.done, 0, sizeof(g.done));
      uint32_t mask = 0;
      for (int32_t s = 0; s < P->n_members; ++s) mask |= (uint32_t)gcall(&g, s) << s;
      const uint32_t ent = P->table[mask];
      if (ent & 2u) {
        d->reason = KW_R_GROUP_EXPR;
      } else if (!(ent & 1u)) {
        d->reason = KW_R_GROUP;
        for (int32_t s = 0; s < P->n_members; ++s)
          if ((ent >> (16 + s)) & 1u) {
            d->causes[d->ncauses++] = s;
            d->arg |= 1ull << s;
          }
        arg16 = P->n_members > 15 ? 0xffffu : (uint32_t)d->arg;
      }
    } else {
      gctx g;
      g.e = e;
      g.G = P;
      g.S = S;
      g.r = r;
      g.zb = zb;
      memset(g.done, 0, sizeof(g.done));
      memset(g.ok, 0, sizeof(g.ok));
      if (!geval(&g, P->n_nodes - 1)) {
        d->reason = KW_R_GROUP;
        for (int32_t s = 0; s < P->n_members && s < ORC_MAX_MEMBERS; ++s)
          if (g.done[s] && !g.ok[s]) {
            d->causes[d->ncauses++] = s;
            if (s < 64) d->arg |= 1ull << s;
          }
        /* more than 15 members: the cause mask lives in the pass's side data */
        arg16 = P->n_members > 15 ? 0xffffu : (uint32_t)d->arg;
      }
    }
  } else {
    fam_out fo = eval_family(e, p, S, r, zb);
    d->reason = fo.reason;
    d->arg = fo.arg;
    d->mutated = fo.mutated;
    arg16 = fo.arg < 0xffffu ? (uint32_t)fo.arg : 0xffffu;
  }
  uint32_t v = (d->reason << 8) | (arg16 << 16);
  int allowed = d->reason == 0;
  if (allowed) v |= KW_V_ALLOWED;
  if (d->mutated) v |= KW_V_MUTATED;
  /* validation_response_with_constraints (service.rs:160-208) for the Validate origin only */
  uint32_t fst = allowed ? KW_FST_NONE : KW_FST_VANILLA;
  int fallowed = allowed;
  if (origin == KW_ORIGIN_VALIDATE) {
    if (P->mode == KW_MODE_MONITOR) {
      fallowed = 1;
      fst = KW_FST_NONE;
    } else if (d->mutated && !P->allowed_to_mutate) {
      fallowed = 0;
      fst = KW_FST_MUTATION_REFUSED;
    }
  }
  if (fallowed) v |= KW_F_ALLOWED;
  if (d->mutated && fst == KW_FST_NONE && (origin == KW_ORIGIN_AUDIT || P->mode == KW_MODE_PROTECT)) v |= KW_F_PATCH;
  v |= fst << KW_F_STATUS_SHIFT;
  d->word = v;
}

static uint32_t verdict(const orc_env *e, int32_t p, const kw_soa *S, uint64_t r, int32_t origin, zbuf *zb) {
  orc_detail d;
  detail(e, p, S, r, origin, zb, &d);
  return d.word;
}

void orc_eval_detail(const orc_env *e, const kw_soa *S, int32_t policy, int32_t origin, uint64_t row, orc_detail *out) {
  zbuf zb;
  zb.big = NULL;
  detail(e, policy, S, row, origin, &zb, out);
  free(zb.big);
}

void orc_eval(const orc_env *e, const kw_soa *S, const int32_t *pols, int32_t npol, int32_t origin,
              uint64_t row0, uint64_t row1, uint32_t *out) {
  zbuf zb;
  zb.big = NULL;
  for (uint64_t r = row0; r < row1; ++r)
    for (int32_t j = 0; j < npol; ++j) out[r * (uint64_t)npol + (uint64_t)j] = verdict(e, pols[j], S, r, origin, &zb);
  free(zb.big);
}

typedef struct {
  const orc_env *e;
  const kw_soa *S;
  const int32_t *pols;
  int32_t npol, origin;
  uint64_t r0, r1;
  uint32_t *out;
  int cpu; /* -1 = not pinned */
} mt_arg;
static void *mt_main(void *a_) {
  mt_arg *a = (mt_arg *)a_;
  if (a->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(a->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  }
  orc_eval(a->e, a->S, a->pols, a->npol, a->origin, a->r0, a->r1, a->out);
  return NULL;
}
void orc_eval_mt(const orc_env *e, const kw_soa *S, const int32_t *pols, int32_t npol,
                 int32_t origin, uint64_t nrows, int threads, uint32_t *out) {
  orc_eval_mt_pinned(e, S, pols, npol, origin, nrows, threads, NULL, out);
}
void orc_eval_mt_pinned(const orc_env *e, const kw_soa *S, const int32_t *pols, int32_t npol, int32_t origin,
                        uint64_t nrows, int threads, const int32_t *cpus, uint32_t *out) {
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  mt_arg *args = (mt_arg *)calloc((size_t)threads, sizeof(mt_arg));
  for (int t = 0; t < threads; ++t) {
    args[t].e = e;
    args[t].S = S;
    args[t].pols = pols;
    args[t].npol = npol;
    args[t].origin = origin;
    args[t].r0 = nrows * (uint64_t)t / (uint64_t)threads;
    args[t].r1 = nrows * (uint64_t)(t + 1) / (uint64_t)threads;
    args[t].out = out;
    args[t].cpu = cpus ? cpus[t] : -1;
    pthread_create(&th[t], NULL, mt_main, &args[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(args);
}
