/*
 * kwregex.c — the oracle's regex matcher. TEST INFRASTRUCTURE ONLY (loaded with kworacle.c by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product).
 *
 * Restates `Regex::new(p)?.is_match(s)` of the Rust `regex` crate for the label constraints of the
 * safe-labels family (constrained_labels; upstream policy absent),
 * in the dialect DESIGN.md §2 fixes: Rust syntax, matching over Unicode scalar values, Rust's
 * Unicode `\d \w \s`, word boundaries and simple case folding (ASCII ones under `(?-u)`; tables:
 * oracle/unicode_data.h), `\p{..}` General_Category classes (r06; other properties refused),
 * back-references / look-around / the R flag refused.
 *
 * Independent of the product's automaton compiler (policy-server_amd/csrc/automaton.cpp, a byte-level
 * DFA built by subset construction): this file parses the pattern itself into a tree over code
 * points, compiles it to a backtracking-free Pike VM program (Thompson's simulation, one thread list
 * per position) and runs it over the subject's code points. tests/test_regex_dialect.py pins it
 * against Python's `re` (a third, independent engine) through a documented translation.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kworacle.h"
#include "unicode_data.h"

/* ------------------------------------------------------------------ code point sets */
typedef struct {
  uint32_t lo, hi;
} crng;
typedef struct {
  crng *r;
  int n, cap;
} cset;

static void cs_push(cset *s, uint32_t lo, uint32_t hi) {
  if (s->n == s->cap) {
    s->cap = s->cap ? 2 * s->cap : 8;
    s->r = (crng *)realloc(s->r, (size_t)s->cap * sizeof(crng));
  }
  s->r[s->n].lo = lo;
  s->r[s->n].hi = hi;
  s->n++;
}
static int crng_cmp(const void *a, const void *b) {
  const crng *x = (const crng *)a, *y = (const crng *)b;
  return x->lo < y->lo ? -1 : x->lo > y->lo ? 1 : 0;
}
static void cs_canon(cset *s) { /* sort and merge overlapping or touching ranges */
  if (s->n < 2) return;
  qsort(s->r, (size_t)s->n, sizeof(crng), crng_cmp);
  int w = 0;
  for (int k = 1; k < s->n; ++k) {
    if (s->r[k].lo <= s->r[w].hi + 1) {
      if (s->r[k].hi > s->r[w].hi) s->r[w].hi = s->r[k].hi;
    } else {
      s->r[++w] = s->r[k];
    }
  }
  s->n = w + 1;
}
static void cs_free(cset *s) {
  free(s->r);
  s->r = NULL;
  s->n = s->cap = 0;
}
static int cs_has(const cset *s, uint32_t c) {
  int lo = 0, hi = s->n - 1;
  while (lo <= hi) {
    int m = (lo + hi) / 2;
    if (c < s->r[m].lo) hi = m - 1;
    else if (c > s->r[m].hi) lo = m + 1;
    else return 1;
  }
  return 0;
}
/* complement within the Unicode scalar values [0, 0xD7FF] u [0xE000, 0x10FFFF] */
static cset cs_complement(const cset *s) {
  cset o = {0};
  uint32_t next = 0;
  for (int k = 0; k < s->n; ++k) {
    if (s->r[k].lo > next) cs_push(&o, next, s->r[k].lo - 1);
    next = s->r[k].hi + 1;
  }
  if (next <= 0x10FFFF) cs_push(&o, next, 0x10FFFF);
  /* cut the surrogates out */
  cset v = {0};
  for (int k = 0; k < o.n; ++k) {
    uint32_t lo = o.r[k].lo, hi = o.r[k].hi;
    if (hi < 0xD800 || lo > 0xDFFF) {
      cs_push(&v, lo, hi);
    } else {
      if (lo < 0xD800) cs_push(&v, lo, 0xD7FF);
      if (hi > 0xDFFF) cs_push(&v, 0xE000, hi);
    }
  }
  cs_free(&o);
  return v;
}
static cset cs_copy(const cset *s) {
  cset o = {0};
  for (int k = 0; k < s->n; ++k) cs_push(&o, s->r[k].lo, s->r[k].hi);
  return o;
}
static void cs_add_all(cset *d, const cset *s) {
  for (int k = 0; k < s->n; ++k) cs_push(d, s->r[k].lo, s->r[k].hi);
  cs_canon(d);
}
static cset cs_and(const cset *a, const cset *b) {
  cset o = {0};
  for (int i = 0; i < a->n; ++i)
    for (int j = 0; j < b->n; ++j) {
      uint32_t lo = a->r[i].lo > b->r[j].lo ? a->r[i].lo : b->r[j].lo;
      uint32_t hi = a->r[i].hi < b->r[j].hi ? a->r[i].hi : b->r[j].hi;
      if (lo <= hi) cs_push(&o, lo, hi);
    }
  cs_canon(&o);
  return o;
}
static cset cs_minus(const cset *a, const cset *b) {
  cset nb = cs_complement(b);
  cset o = cs_and(a, &nb);
  cs_free(&nb);
  return o;
}
/* ASCII simple case folding: add the other case of every ASCII letter in the set */
static void cs_casefold_ascii(cset *s) {
  int n = s->n;
  for (int k = 0; k < n; ++k) {
    for (uint32_t c = s->r[k].lo; c <= s->r[k].hi && c <= 'z'; ++c) {
      if (c >= 'A' && c <= 'Z') cs_push(s, c + 32, c + 32);
      else if (c >= 'a' && c <= 'z') cs_push(s, c - 32, c - 32);
    }
  }
  cs_canon(s);
}
static int cs_beyond_ascii(const cset *s) { return s->n > 0 && s->r[s->n - 1].hi > 0x7F; }

static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return x < y ? -1 : x > y;
}
/* Unicode simple case folding: the set of folds its members have, then every code point whose
   fold is one of them (orc_uni_fold: (code point, fold) pairs of the non-trivial orbits) */
static void cs_casefold_unicode(cset *s) {
  uint32_t *keys = (uint32_t *)malloc(ORC_UNI_FOLD_N * sizeof(uint32_t));
  size_t nk = 0;
  for (size_t k = 0; k < ORC_UNI_FOLD_N; ++k)
    if (cs_has(s, orc_uni_fold[2 * k])) keys[nk++] = orc_uni_fold[2 * k + 1];
  qsort(keys, nk, sizeof(uint32_t), cmp_u32);
  for (size_t k = 0; k < ORC_UNI_FOLD_N; ++k) {
    uint32_t f = orc_uni_fold[2 * k + 1];
    if (nk && bsearch(&f, keys, nk, sizeof(uint32_t), cmp_u32)) cs_push(s, orc_uni_fold[2 * k], orc_uni_fold[2 * k]);
  }
  free(keys);
  cs_canon(s);
}
static void cs_casefold_mode(cset *s, int unicode) {
  if (unicode) cs_casefold_unicode(s);
  else cs_casefold_ascii(s);
}
#define cs_casefold(s) cs_casefold_mode((s), P->fl.u)
/* the Unicode classes of \d \w \s (Rust regex: Nd; Alphabetic + M + Nd + Pc + Join_Control;
   White_Space) */
static void uni_class(char which, cset *out) {
  memset(out, 0, sizeof(*out));
  if (which == 's') {
    static const uint32_t ws[] = {9, 13, 0x20, 0x20, 0x85, 0x85, 0xA0, 0xA0, 0x1680, 0x1680, 0x2000, 0x200A,
                                  0x2028, 0x2029, 0x202F, 0x202F, 0x205F, 0x205F, 0x3000, 0x3000};
    for (size_t k = 0; k < sizeof(ws) / sizeof(ws[0]); k += 2) cs_push(out, ws[k], ws[k + 1]);
  } else {
    const uint32_t *t = which == 'd' ? orc_uni_digit : orc_uni_word;
    size_t n = which == 'd' ? ORC_UNI_DIGIT_N : ORC_UNI_WORD_N;
    for (size_t k = 0; k < n; ++k) cs_push(out, t[2 * k], t[2 * k + 1]);
  }
  cs_canon(out);
}

/* \p{..} (r06): a General_Category value, matched loosely as regex-syntax's symbolic_name_normalize
   (ASCII letters lowercased; ' ', '_', '-' and non-ASCII bytes dropped; a leading "is" dropped, but
   "isc" stays), bare or after gc= / general_category=; Any, ASCII, Assigned; White_Space. 1 = a set
   in *out, 0 = not supported */
static void gc_norm(const char *s, size_t n, char *out) {
  size_t at = 0, k = 0;
  int is = n >= 2 && (s[0] | 0x20) == 'i' && (s[1] | 0x20) == 's';
  if (is) k = 2;
  for (; k < n; ++k) {
    unsigned char b = (unsigned char)s[k];
    if (b == ' ' || b == '_' || b == '-' || b >= 0x80) continue;
    out[at++] = (char)(b >= 'A' && b <= 'Z' ? b + 32 : b);
  }
  out[at] = 0;
  if (is && !strcmp(out, "c")) strcpy(out, "isc");
}
static int gc_value_set(const char *v, cset *out) {
  static const char *const names[][2] = {
      {"lu", "Lu"}, {"uppercaseletter", "Lu"}, {"ll", "Ll"}, {"lowercaseletter", "Ll"}, {"lt", "Lt"},
      {"titlecaseletter", "Lt"}, {"lc", "LC"}, {"casedletter", "LC"}, {"l&", "LC"}, {"lm", "Lm"},
      {"modifierletter", "Lm"}, {"lo", "Lo"}, {"otherletter", "Lo"}, {"l", "L"}, {"letter", "L"},
      {"mn", "Mn"}, {"nonspacingmark", "Mn"}, {"mc", "Mc"}, {"spacingmark", "Mc"}, {"me", "Me"},
      {"enclosingmark", "Me"}, {"m", "M"}, {"mark", "M"}, {"combiningmark", "M"}, {"nd", "Nd"},
      {"decimalnumber", "Nd"}, {"digit", "Nd"}, {"nl", "Nl"}, {"letternumber", "Nl"}, {"no", "No"},
      {"othernumber", "No"}, {"n", "N"}, {"number", "N"}, {"pc", "Pc"}, {"connectorpunctuation", "Pc"},
      {"pd", "Pd"}, {"dashpunctuation", "Pd"}, {"ps", "Ps"}, {"openpunctuation", "Ps"}, {"pe", "Pe"},
      {"closepunctuation", "Pe"}, {"pi", "Pi"}, {"initialpunctuation", "Pi"}, {"pf", "Pf"},
      {"finalpunctuation", "Pf"}, {"po", "Po"}, {"otherpunctuation", "Po"}, {"p", "P"}, {"punctuation", "P"},
      {"punct", "P"}, {"sm", "Sm"}, {"mathsymbol", "Sm"}, {"sc", "Sc"}, {"currencysymbol", "Sc"},
      {"sk", "Sk"}, {"modifiersymbol", "Sk"}, {"so", "So"}, {"othersymbol", "So"}, {"s", "S"},
      {"symbol", "S"}, {"zs", "Zs"}, {"spaceseparator", "Zs"}, {"zl", "Zl"}, {"lineseparator", "Zl"},
      {"zp", "Zp"}, {"paragraphseparator", "Zp"}, {"z", "Z"}, {"separator", "Z"}, {"cc", "Cc"},
      {"control", "Cc"}, {"cntrl", "Cc"}, {"cf", "Cf"}, {"format", "Cf"}, {"cs", "Cs"}, {"surrogate", "Cs"},
      {"co", "Co"}, {"privateuse", "Co"}, {"cn", "Cn"}, {"unassigned", "Cn"}, {"c", "C"}, {"other", "C"},
      {"any", "Any"}, {"ascii", "ASCII"}, {"assigned", "Assigned"}};
  const char *g = NULL;
  for (size_t k = 0; k < sizeof(names) / sizeof(names[0]); ++k)
    if (!strcmp(v, names[k][0])) g = names[k][1];
  if (!g) return 0;
  memset(out, 0, sizeof(*out));
  if (!strcmp(g, "Any")) {
    cs_push(out, 0, 0x10FFFF);
  } else if (!strcmp(g, "ASCII")) {
    cs_push(out, 0, 0x7F);
  } else {
    /* the runs of every category the value covers; the unassigned code points are the gaps */
    cset assigned = {0};
    for (size_t k = 0; k < ORC_UNI_GC_N; ++k) {
      const char *c = ORC_GC_NAMES[orc_uni_gc[3 * k + 2]];
      int take;
      if (!strcmp(g, "LC")) take = !strcmp(c, "Lu") || !strcmp(c, "Ll") || !strcmp(c, "Lt");
      else if (g[1] == 0) take = c[0] == g[0];
      else take = !strcmp(c, g);
      cs_push(&assigned, orc_uni_gc[3 * k], orc_uni_gc[3 * k + 1]);
      if (take && strcmp(g, "Assigned")) cs_push(out, orc_uni_gc[3 * k], orc_uni_gc[3 * k + 1]);
    }
    cs_canon(&assigned);
    if (!strcmp(g, "Assigned")) {
      cs_add_all(out, &assigned);
    } else if (!strcmp(g, "Cn") || !strcmp(g, "C")) {
      cset gaps = cs_complement(&assigned); /* (surrogates excluded by the complement) */
      cs_add_all(out, &gaps);
      cs_free(&gaps);
    }
    cs_free(&assigned);
  }
  /* scalar values only: intersect with the complement of the empty set */
  cs_canon(out);
  cset none = {0}, all = cs_complement(&none);
  cset v2 = cs_and(out, &all);
  cs_free(&all);
  cs_free(out);
  *out = v2;
  return 1;
}
static int unicode_property(const char *body, size_t n, cset *out, int *negate) {
  char prop[128], val[128];
  const char *eq = memchr(body, '=', n);
  if (!eq) eq = memchr(body, ':', n);
  if (n >= sizeof(val)) return 0;
  if (eq) {
    size_t pn = (size_t)(eq - body);
    if (pn && body[pn - 1] == '!') {
      *negate = !*negate;
      --pn;
    }
    gc_norm(body, pn, prop);
    if (strcmp(prop, "gc") && strcmp(prop, "generalcategory")) return 0;
    gc_norm(eq + 1, n - (size_t)(eq + 1 - body), val);
  } else {
    gc_norm(body, n, val);
    if (!strcmp(val, "whitespace") || !strcmp(val, "wspace") || !strcmp(val, "space")) {
      uni_class('s', out);
      return 1;
    }
  }
  return gc_value_set(val, out);
}

/* the ASCII classes ([:name:], \d \w \s) */
static int named_class(const char *name, size_t len, cset *out) {
  static const struct {
    const char *name;
    const char *ranges; /* pairs of bytes */
  } tab[] = {
      {"alnum", "09AZaz"}, {"alpha", "AZaz"},     {"ascii", "\x01\x7f"}, {"blank", "\t\t  "},
      {"cntrl", "\x01\x1f\x7f\x7f"}, {"digit", "09"}, {"graph", "!~"},   {"lower", "az"},
      {"print", " ~"},     {"punct", "!/:@[`{~"}, {"space", "\t\r  "},   {"upper", "AZ"},
      {"word", "09AZ__az"}, {"xdigit", "09AFaf"},
  };
  for (size_t t = 0; t < sizeof(tab) / sizeof(tab[0]); ++t) {
    if (strlen(tab[t].name) != len || memcmp(tab[t].name, name, len) != 0) continue;
    memset(out, 0, sizeof(*out));
    for (const char *r = tab[t].ranges; *r; r += 2) cs_push(out, (unsigned char)r[0], (unsigned char)r[1]);
    if (!strcmp(tab[t].name, "ascii") || !strcmp(tab[t].name, "cntrl")) cs_push(out, 0, 0); /* NUL */
    cs_canon(out);
    return 1;
  }
  return 0;
}

/* ------------------------------------------------------------------ syntax tree */
enum { N_EMPTY, N_SET, N_CAT, N_ALT, N_REP, N_ASSERT };
enum { A_TEXT_START, A_TEXT_END, A_LINE_START, A_LINE_END, A_WORD, A_NOT_WORD, A_WORD_START, A_WORD_END,
       A_WORD_START_HALF, A_WORD_END_HALF };
#define A_UNI 0x100 /* a word boundary over Unicode word characters */
typedef struct {
  int kind;
  cset set;
  int a, b;
  int min, max; /* N_REP, max < 0: unbounded */
  int akind;
} rnode;

typedef struct {
  int i, m, s, x, u;
} rflags;

typedef struct {
  const char *p;
  size_t n, at;
  rnode *nodes;
  int nn, ncap;
  char err[160];
  rflags fl;
  char **names;
  int nnames;
  int depth;
} rparse;

static int new_node(rparse *P, int kind) {
  if (P->nn == P->ncap) {
    P->ncap = P->ncap ? 2 * P->ncap : 32;
    P->nodes = (rnode *)realloc(P->nodes, (size_t)P->ncap * sizeof(rnode));
  }
  memset(&P->nodes[P->nn], 0, sizeof(rnode));
  P->nodes[P->nn].kind = kind;
  P->nodes[P->nn].a = P->nodes[P->nn].b = -1;
  return P->nn++;
}
static int bad(rparse *P, const char *msg) {
  if (!P->err[0]) snprintf(P->err, sizeof(P->err), "%s", msg);
  return -1;
}
static int at_end(const rparse *P) { return P->at >= P->n; }
static int peek(const rparse *P) { return at_end(P) ? -1 : (unsigned char)P->p[P->at]; }

/* next UTF-8 character of the pattern, -1 when malformed */
static int64_t next_char(rparse *P) {
  const unsigned char *s = (const unsigned char *)P->p + P->at;
  size_t left = P->n - P->at;
  uint32_t c = s[0];
  int len = 1;
  if (c >= 0x80) {
    if ((c & 0xE0) == 0xC0) len = 2, c &= 0x1F;
    else if ((c & 0xF0) == 0xE0) len = 3, c &= 0x0F;
    else if ((c & 0xF8) == 0xF0) len = 4, c &= 0x07;
    else return -1;
    if ((size_t)len > left) return -1;
    for (int k = 1; k < len; ++k) {
      if ((s[k] & 0xC0) != 0x80) return -1;
      c = (c << 6) | (s[k] & 0x3F);
    }
    if ((len == 2 && c < 0x80) || (len == 3 && c < 0x800) || (len == 4 && c < 0x10000) || c > 0x10FFFF ||
        (c >= 0xD800 && c <= 0xDFFF))
      return -1;
  }
  P->at += (size_t)len;
  return c;
}
static int uni_space(uint32_t c) { /* char::is_whitespace */
  return (c >= 9 && c <= 13) || c == 32 || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
         c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
static void skip_verbose(rparse *P) { /* flag x: white space and # comments */
  if (!P->fl.x) return;
  while (!at_end(P)) {
    size_t save = P->at;
    int64_t c = next_char(P);
    if (c == '#') {
      while (!at_end(P) && P->p[P->at] != '\n') P->at++;
    } else if (c < 0 || !uni_space((uint32_t)c)) {
      P->at = save;
      return;
    }
  }
}

static int parse_alt(rparse *P);

static int set_leaf(rparse *P, cset s, int fold) {
  if (fold && P->fl.i) cs_casefold(&s);
  if (!P->fl.u && cs_beyond_ascii(&s)) {
    cs_free(&s);
    return bad(P, "non-ASCII match with Unicode mode off");
  }
  int k = new_node(P, N_SET);
  P->nodes[k].set = s;
  return k;
}
static int assert_leaf(rparse *P, int kind) {
  int k = new_node(P, N_ASSERT);
  P->nodes[k].akind = kind;
  return k;
}

static int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
/* \x \u \U: a fixed number of digits or {1 to 8 digits}; -1 when invalid */
static int64_t parse_hex(rparse *P, int digits) {
  uint64_t v = 0;
  if (peek(P) == '{') {
    P->at++;
    int nd = 0;
    while (!at_end(P) && peek(P) != '}') {
      int h = hexval(peek(P));
      if (h < 0 || nd == 8) return -1;
      v = v * 16 + (uint64_t)h;
      nd++;
      P->at++;
    }
    if (at_end(P) || nd == 0) return -1;
    P->at++;
  } else {
    for (int k = 0; k < digits; ++k) {
      int h = at_end(P) ? -1 : hexval(peek(P));
      if (h < 0) return -1;
      v = v * 16 + (uint64_t)h;
      P->at++;
    }
  }
  if (v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return -1;
  return (int64_t)v;
}

/* escape after '\': 1 = a set in *out (*single = its code point when it is one character that may
   bound a range, else -1), 2 = an assertion in *akind, 0 = error */
static int parse_escape(rparse *P, int in_class, cset *out, int64_t *single, int *akind) {
  memset(out, 0, sizeof(*out));
  *single = -1;
  if (at_end(P)) return bad(P, "incomplete escape"), 0;
  int64_t c = next_char(P);
  if (c < 0) return bad(P, "bad UTF-8"), 0;
  const char *cls = NULL;
  int negate = 0;
  switch (c) {
  case 'd': cls = "digit"; break;
  case 'D': cls = "digit"; negate = 1; break;
  case 'w': cls = "word"; break;
  case 'W': cls = "word"; negate = 1; break;
  case 's': cls = "space"; break;
  case 'S': cls = "space"; negate = 1; break;
  default: break;
  }
  if (cls) {
    if (P->fl.u) uni_class(cls[0], out);
    else named_class(cls, strlen(cls), out);
    if (negate) {
      cset n = cs_complement(out);
      cs_free(out);
      *out = n;
    }
    return 1;
  }
  uint32_t lit = 0;
  int have = 1;
  switch (c) {
  case 'a': lit = 7; break;
  case 'f': lit = 12; break;
  case 't': lit = 9; break;
  case 'n': lit = 10; break;
  case 'r': lit = 13; break;
  case 'v': lit = 11; break;
  case 'x':
  case 'u':
  case 'U': {
    int64_t v = parse_hex(P, c == 'x' ? 2 : c == 'u' ? 4 : 8);
    if (v < 0) return bad(P, "bad hex escape"), 0;
    if (!P->fl.u && v > 0x7F) return bad(P, "non-ASCII escape with Unicode mode off"), 0;
    lit = (uint32_t)v;
    break;
  }
  default: have = 0; break;
  }
  if (!have) {
    if (c == 'p' || c == 'P') {
      if (!P->fl.u) return bad(P, "Unicode class with Unicode mode off"), 0;
      const char *body = P->p + P->at;
      size_t n;
      if (peek(P) == '{') {
        const char *e = memchr(body, '}', P->n - P->at);
        if (!e) return bad(P, "unclosed Unicode class"), 0;
        ++body;
        n = (size_t)(e - body);
        P->at += n + 2;
      } else {
        if (at_end(P)) return bad(P, "incomplete Unicode class"), 0;
        int64_t l = next_char(P);
        if (l < 0 || l >= 0x80) return bad(P, "bad Unicode class name"), 0;
        n = 1;
      }
      int negate = c == 'P';
      if (!unicode_property(body, n, out, &negate)) return bad(P, "Unicode property outside this dialect"), 0;
      if (P->fl.i) cs_casefold(out); /* regex-syntax folds a Unicode class before negating it */
      if (negate) {
        cset neg = cs_complement(out);
        cs_free(out);
        *out = neg;
      }
      return 1;
    }
    if (!in_class) {
      int k = -1;
      if (c == 'A') k = A_TEXT_START;
      else if (c == 'z') k = A_TEXT_END;
      else if (c == 'B') {
        if (!P->fl.u) return bad(P, "ASCII \\B can match inside a code point"), 0; /* regex-syntax InvalidUtf8 */
        k = A_NOT_WORD;
      }
      else if (c == '<') k = A_WORD_START;
      else if (c == '>') k = A_WORD_END;
      else if (c == 'b') {
        k = A_WORD;
        if (peek(P) == '{') {
          static const struct {
            const char *w;
            int k;
          } bw[] = {{"{start}", A_WORD_START}, {"{end}", A_WORD_END}, {"{start-half}", A_WORD_START_HALF},
                    {"{end-half}", A_WORD_END_HALF}};
          k = -1;
          for (int t = 0; t < 4; ++t) {
            size_t L = strlen(bw[t].w);
            if (P->n - P->at >= L && memcmp(P->p + P->at, bw[t].w, L) == 0) {
              k = bw[t].k;
              P->at += L;
              break;
            }
          }
          if (k < 0) return bad(P, "bad word boundary"), 0;
        }
      }
      if (k >= 0) {
        /* word boundaries in Unicode mode read Unicode word characters */
        if (P->fl.u && k != A_TEXT_START && k != A_TEXT_END) k |= A_UNI;
        *akind = k;
        return 2;
      }
    }
    int alnum = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
    if (c >= 0x80 || alnum || c == '<' || c == '>') return bad(P, "unknown escape"), 0;
    lit = (uint32_t)c; /* escaped ASCII punctuation or space */
  }
  cs_push(out, lit, lit);
  *single = lit;
  return 1;
}

/* ---- bracket classes */
static int class_expr(rparse *P, cset *out);

static int set_op_here(const rparse *P) {
  if (P->n - P->at < 2) return 0;
  char a = P->p[P->at], b = P->p[P->at + 1];
  if (a == b && (a == '&' || a == '-' || a == '~')) return a;
  return 0;
}

/* a class primitive: nested class, [:name:], escape or character */
static int class_atom(rparse *P, cset *out, int64_t *single) {
  *single = -1;
  memset(out, 0, sizeof(*out));
  if (peek(P) == '[') {
    if (P->at + 1 < P->n && P->p[P->at + 1] == ':') {
      const char *end = strstr(P->p + P->at + 2, ":]");
      if (end && (size_t)(end - P->p) < P->n) {
        const char *nm = P->p + P->at + 2;
        size_t len = (size_t)(end - nm);
        int neg = len > 0 && nm[0] == '^';
        if (named_class(nm + neg, len - (size_t)neg, out)) {
          P->at = (size_t)(end - P->p) + 2;
          if (P->fl.i) cs_casefold(out);
          if (neg) {
            cset c = cs_complement(out);
            cs_free(out);
            *out = c;
          }
          return 1;
        }
      }
    }
    P->at++;
    return class_expr(P, out);
  }
  if (peek(P) == '\\') {
    P->at++;
    int ak;
    int r = parse_escape(P, 1, out, single, &ak);
    if (r != 1) return 0;
    if (P->fl.i) cs_casefold(out);
    return 1;
  }
  int64_t c = next_char(P);
  if (c < 0) return bad(P, "bad UTF-8"), 0;
  cs_push(out, (uint32_t)c, (uint32_t)c);
  *single = c;
  if (P->fl.i) cs_casefold(out);
  return 1;
}

/* juxtaposed items (with ranges) until ']' or a set operator */
static int class_items(rparse *P, cset *acc, int leading_bracket_literal) {
  int count = 0;
  memset(acc, 0, sizeof(*acc));
  for (;;) {
    skip_verbose(P);
    if (at_end(P)) return bad(P, "unclosed class"), 0;
    if (peek(P) == ']' && !(leading_bracket_literal && count == 0)) break;
    if (count > 0 && set_op_here(P)) break;
    cset item;
    int64_t lo;
    if (peek(P) == ']') { /* leading ']' */
      P->at++;
      memset(&item, 0, sizeof(item));
      cs_push(&item, ']', ']');
      lo = ']';
    } else if (!class_atom(P, &item, &lo)) {
      return 0;
    }
    skip_verbose(P);
    if (lo >= 0 && peek(P) == '-' && P->at + 1 < P->n && P->p[P->at + 1] != ']' && !set_op_here(P)) {
      P->at++;
      skip_verbose(P);
      if (at_end(P) || peek(P) == '[') return bad(P, "bad range"), 0;
      cset hs;
      int64_t hi;
      if (!class_atom(P, &hs, &hi)) return 0;
      cs_free(&hs);
      if (hi < 0 || hi < lo) return bad(P, "bad range"), 0;
      cs_free(&item);
      cs_push(&item, (uint32_t)lo, (uint32_t)hi);
      if (P->fl.i) cs_casefold(&item);
    }
    cs_add_all(acc, &item);
    cs_free(&item);
    count++;
  }
  if (!count) return bad(P, "empty class"), 0;
  return 1;
}

/* after '[': [^] items (op items)* ']' */
static int class_expr(rparse *P, cset *out) {
  int neg = 0;
  skip_verbose(P);
  if (peek(P) == '^') {
    neg = 1;
    P->at++;
  }
  cset acc;
  if (!class_items(P, &acc, 1)) return 0;
  for (;;) {
    skip_verbose(P);
    int op = set_op_here(P);
    if (!op) break;
    P->at += 2;
    cset rhs, r;
    if (!class_items(P, &rhs, 0)) return 0;
    if (op == '&') {
      r = cs_and(&acc, &rhs);
    } else if (op == '-') {
      r = cs_minus(&acc, &rhs);
    } else {
      cset x = cs_minus(&acc, &rhs), y = cs_minus(&rhs, &acc);
      cs_add_all(&x, &y);
      cs_free(&y);
      r = x;
    }
    cs_free(&acc);
    cs_free(&rhs);
    acc = r;
  }
  if (peek(P) != ']') return bad(P, "unclosed class"), 0;
  P->at++;
  if (neg) {
    cset c = cs_complement(&acc);
    cs_free(&acc);
    acc = c;
  }
  *out = acc;
  return 1;
}

/* ---- groups, atoms, repetition, concatenation */
static int group_rest(rparse *P, rflags inner) {
  rflags outer = P->fl;
  P->fl = inner;
  if (++P->depth > 250) return bad(P, "nested too deeply");
  int r = parse_alt(P);
  P->depth--;
  P->fl = outer;
  if (r < 0) return -1;
  if (peek(P) != ')') return bad(P, "unclosed group");
  P->at++;
  return r;
}

/* -2: a flag directive "(?flags)" (no node) */
static int parse_atom(rparse *P) {
  int c = peek(P);
  if (c == '(') {
    P->at++;
    if (peek(P) != '?') return group_rest(P, P->fl);
    P->at++;
    if (peek(P) == ':') {
      P->at++;
      return group_rest(P, P->fl);
    }
    if (peek(P) == 'P' || peek(P) == '<') {
      if (peek(P) == 'P') {
        P->at++;
        if (peek(P) != '<') return bad(P, "bad group");
      }
      P->at++;
      size_t s0 = P->at;
      while (!at_end(P) && peek(P) != '>') {
        int x = peek(P);
        int ok = x == '_' || (x >= 'a' && x <= 'z') || (x >= 'A' && x <= 'Z') ||
                 (P->at > s0 && ((x >= '0' && x <= '9') || x == '.' || x == '[' || x == ']'));
        if (!ok) return bad(P, "bad group name");
        P->at++;
      }
      if (at_end(P) || P->at == s0) return bad(P, "bad group name");
      size_t len = P->at - s0;
      for (int k = 0; k < P->nnames; ++k)
        if (strlen(P->names[k]) == len && !memcmp(P->names[k], P->p + s0, len)) return bad(P, "duplicate group name");
      P->names = (char **)realloc(P->names, (size_t)(P->nnames + 1) * sizeof(char *));
      P->names[P->nnames] = (char *)calloc(len + 1, 1);
      memcpy(P->names[P->nnames++], P->p + s0, len);
      P->at++;
      return group_rest(P, P->fl);
    }
    /* flags */
    rflags f = P->fl;
    int negating = 0, any = 0, since_neg = 0;
    char seen[16] = {0};
    int nseen = 0;
    while (!at_end(P) && peek(P) != ':' && peek(P) != ')') {
      int x = P->p[P->at++];
      if (x == '-') {
        if (negating) return bad(P, "double negation");
        negating = 1;
        since_neg = 0;
        continue;
      }
      if (memchr(seen, x, (size_t)nseen)) return bad(P, "repeated flag");
      if (nseen < 15) seen[nseen++] = (char)x;
      int on = !negating;
      if (x == 'i') f.i = on;
      else if (x == 'm') f.m = on;
      else if (x == 's') f.s = on;
      else if (x == 'x') f.x = on;
      else if (x == 'u') f.u = on;
      else if (x == 'U') { /* greed: no effect on is_match */ }
      else return bad(P, x == 'R' ? "CRLF flag unsupported" : "unknown flag");
      any = 1;
      since_neg = negating;
    }
    if (at_end(P)) return bad(P, "unclosed group");
    if (!any || (negating && !since_neg)) return bad(P, "bad flags");
    if (P->p[P->at++] == ')') {
      P->fl = f;
      return -2;
    }
    return group_rest(P, f);
  }
  if (c == '*' || c == '+' || c == '?' || c == '{') return bad(P, "nothing to repeat");
  if (c == '^') {
    P->at++;
    return assert_leaf(P, P->fl.m ? A_LINE_START : A_TEXT_START);
  }
  if (c == '$') {
    P->at++;
    return assert_leaf(P, P->fl.m ? A_LINE_END : A_TEXT_END);
  }
  if (c == '.') {
    P->at++;
    cset s = {0};
    if (!P->fl.s) cs_push(&s, '\n', '\n');
    cset all = cs_complement(&s);
    cs_free(&s);
    if (!P->fl.u) {
      cs_free(&all);
      return bad(P, "'.' with Unicode mode off");
    }
    return set_leaf(P, all, 0);
  }
  if (c == '[') {
    P->at++;
    cset s;
    if (!class_expr(P, &s)) return -1;
    cset valid = {0}, cut;
    cs_push(&valid, 0, 0xD7FF);
    cs_push(&valid, 0xE000, 0x10FFFF);
    cut = cs_and(&s, &valid);
    cs_free(&s);
    cs_free(&valid);
    return set_leaf(P, cut, 0);
  }
  if (c == '\\') {
    P->at++;
    cset s;
    int64_t single;
    int ak;
    int r = parse_escape(P, 0, &s, &single, &ak);
    if (r == 0) return -1;
    if (r == 2) return assert_leaf(P, ak);
    return set_leaf(P, s, 1);
  }
  int64_t ch = next_char(P);
  if (ch < 0) return bad(P, "bad UTF-8");
  cset s = {0};
  cs_push(&s, (uint32_t)ch, (uint32_t)ch);
  if (P->fl.i) cs_casefold(&s);
  int k = new_node(P, N_SET); /* a literal character: allowed with Unicode mode off, whatever it is */
  P->nodes[k].set = s;
  return k;
}

static int read_count(rparse *P, int *v) {
  skip_verbose(P);
  long x = 0;
  int nd = 0;
  while (!at_end(P) && peek(P) >= '0' && peek(P) <= '9') {
    x = x * 10 + (peek(P) - '0');
    if (x > 100000) return 0;
    P->at++;
    nd++;
  }
  skip_verbose(P);
  *v = (int)x;
  return nd > 0;
}

static int parse_repeat(rparse *P) {
  int a = parse_atom(P);
  if (a < 0) return a;
  for (;;) {
    skip_verbose(P);
    int c = peek(P), mn, mx;
    if (c == '*') mn = 0, mx = -1;
    else if (c == '+') mn = 1, mx = -1;
    else if (c == '?') mn = 0, mx = 1;
    else if (c == '{') {
      P->at++;
      if (!read_count(P, &mn)) return bad(P, "bad repetition");
      mx = mn;
      if (peek(P) == ',') {
        P->at++;
        skip_verbose(P);
        if (peek(P) == '}') mx = -1;
        else if (!read_count(P, &mx) || mx < mn) return bad(P, "bad repetition");
      }
      if (peek(P) != '}') return bad(P, "bad repetition");
    } else {
      break;
    }
    P->at++;
    if (peek(P) == '?') P->at++; /* non-greedy */
    int r = new_node(P, N_REP);
    P->nodes[r].a = a;
    P->nodes[r].min = mn;
    P->nodes[r].max = mx;
    a = r;
  }
  return a;
}

static int parse_concat(rparse *P) {
  int acc = new_node(P, N_EMPTY);
  for (;;) {
    skip_verbose(P);
    if (at_end(P) || peek(P) == '|' || peek(P) == ')') return acc;
    int r = parse_repeat(P);
    if (r == -2) continue;
    if (r < 0) return -1;
    int k = new_node(P, N_CAT);
    P->nodes[k].a = acc;
    P->nodes[k].b = r;
    acc = k;
  }
}

static int parse_alt(rparse *P) {
  int l = parse_concat(P);
  if (l < 0) return -1;
  while (peek(P) == '|') {
    P->at++;
    int r = parse_concat(P);
    if (r < 0) return -1;
    int k = new_node(P, N_ALT);
    P->nodes[k].a = l;
    P->nodes[k].b = r;
    l = k;
  }
  return l;
}

/* ------------------------------------------------------------------ Pike VM program */
enum { I_SET, I_SPLIT, I_JMP, I_ASSERT, I_MATCH };
typedef struct {
  int op, x, y; /* I_SET: x = set index; I_SPLIT: x, y; I_JMP: x; I_ASSERT: x = kind */
} rinst;

struct orc_re {
  rinst *code;
  int ncode, cap;
  cset *sets;
  int nsets;
  int too_big;
};

static int emit(orc_re *R, int op, int x, int y) {
  if (R->ncode >= 2000000) {
    R->too_big = 1;
    return R->ncode;
  }
  if (R->ncode == R->cap) {
    R->cap = R->cap ? 2 * R->cap : 64;
    R->code = (rinst *)realloc(R->code, (size_t)R->cap * sizeof(rinst));
  }
  R->code[R->ncode].op = op;
  R->code[R->ncode].x = x;
  R->code[R->ncode].y = y;
  return R->ncode++;
}

static void gen(orc_re *R, rparse *P, int k) {
  if (R->too_big) return;
  rnode *nd = &P->nodes[k];
  switch (nd->kind) {
  case N_EMPTY: break;
  case N_SET: {
    R->sets = (cset *)realloc(R->sets, (size_t)(R->nsets + 1) * sizeof(cset));
    R->sets[R->nsets] = cs_copy(&nd->set);
    emit(R, I_SET, R->nsets++, 0);
    break;
  }
  case N_ASSERT: emit(R, I_ASSERT, nd->akind, 0); break;
  case N_CAT:
    gen(R, P, nd->a);
    gen(R, P, P->nodes[k].b);
    break;
  case N_ALT: {
    int sp = emit(R, I_SPLIT, 0, 0);
    R->code[sp].x = R->ncode;
    gen(R, P, nd->a);
    int j = emit(R, I_JMP, 0, 0);
    if (R->too_big) return;
    R->code[sp].y = R->ncode;
    gen(R, P, P->nodes[k].b);
    if (R->too_big) return;
    R->code[j].x = R->ncode;
    break;
  }
  case N_REP: {
    int a = nd->a, mn = nd->min, mx = nd->max;
    for (int t = 0; t < mn; ++t) gen(R, P, a);
    if (mx < 0) { /* L: split body, out; body; jmp L */
      int L = emit(R, I_SPLIT, 0, 0);
      R->code[L].x = R->ncode;
      gen(R, P, a);
      emit(R, I_JMP, L, 0);
      if (R->too_big) return;
      R->code[L].y = R->ncode;
    } else {
      int pend[1024], np = 0;
      int *pv = mx - mn > 1024 ? (int *)malloc((size_t)(mx - mn) * sizeof(int)) : pend;
      for (int t = mn; t < mx; ++t) {
        int sp = emit(R, I_SPLIT, 0, 0);
        if (R->too_big) break;
        R->code[sp].x = R->ncode;
        pv[np++] = sp;
        gen(R, P, a);
      }
      if (!R->too_big)
        for (int t = 0; t < np; ++t) R->code[pv[t]].y = R->ncode;
      if (pv != pend) free(pv);
    }
    break;
  }
  }
}

static void free_parse(rparse *P) {
  for (int k = 0; k < P->nn; ++k) cs_free(&P->nodes[k].set);
  free(P->nodes);
  for (int k = 0; k < P->nnames; ++k) free(P->names[k]);
  free(P->names);
}

orc_re *orc_re_compile(const char *pattern, char *err, int errlen) {
  rparse P;
  memset(&P, 0, sizeof(P));
  P.p = pattern;
  P.n = strlen(pattern);
  P.fl.u = 1;
  int root = parse_alt(&P);
  if (root >= 0 && !at_end(&P)) root = bad(&P, "unopened group");
  if (root < 0) {
    if (err && errlen > 0) snprintf(err, (size_t)errlen, "%s", P.err);
    free_parse(&P);
    return NULL;
  }
  orc_re *R = (orc_re *)calloc(1, sizeof(orc_re));
  gen(R, &P, root);
  emit(R, I_MATCH, 0, 0);
  free_parse(&P);
  if (R->too_big) {
    if (err && errlen > 0) snprintf(err, (size_t)errlen, "regular expression too large");
    orc_re_free(R);
    return NULL;
  }
  return R;
}

void orc_re_free(orc_re *R) {
  if (!R) return;
  for (int k = 0; k < R->nsets; ++k) cs_free(&R->sets[k]);
  free(R->sets);
  free(R->code);
  free(R);
}

/* ------------------------------------------------------------------ matching */
static int is_word_cp(int64_t c, int unicode) {
  if (c >= 0 && c < 0x80)
    return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
  if (!unicode || c < 0 || c > 0x10FFFF) return 0;
  size_t lo = 0, hi = ORC_UNI_WORD_N;
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (orc_uni_word[2 * m + 1] < (uint32_t)c) lo = m + 1;
    else hi = m;
  }
  return lo < ORC_UNI_WORD_N && orc_uni_word[2 * lo] <= (uint32_t)c;
}
static int assert_holds(int kind, int64_t prev, int64_t next) { /* -1: start / end of the text */
  int uni = (kind & A_UNI) != 0;
  int wp = is_word_cp(prev, uni), wn = is_word_cp(next, uni);
  switch (kind & ~A_UNI) {
  case A_TEXT_START: return prev < 0;
  case A_TEXT_END: return next < 0;
  case A_LINE_START: return prev < 0 || prev == '\n';
  case A_LINE_END: return next < 0 || next == '\n';
  case A_WORD: return wp != wn;
  case A_NOT_WORD: return wp == wn;
  case A_WORD_START: return !wp && wn;
  case A_WORD_END: return wp && !wn;
  case A_WORD_START_HALF: return !wp;
  case A_WORD_END_HALF: return !wn;
  }
  return 0;
}

typedef struct {
  int *pc;
  int n;
} tlist;

/* add the thread `pc0` at position i (prev / next code points) with its epsilon closure */
static int add_thread(const orc_re *R, tlist *L, uint32_t *mark, uint32_t gen_, int *stack, int pc0, int64_t prev,
                      int64_t next) {
  int sp = 0, matched = 0;
  stack[sp++] = pc0;
  while (sp) {
    int pc = stack[--sp];
    if (mark[pc] == gen_) continue;
    mark[pc] = gen_;
    const rinst *in = &R->code[pc];
    switch (in->op) {
    case I_JMP: stack[sp++] = in->x; break;
    case I_SPLIT:
      stack[sp++] = in->y;
      stack[sp++] = in->x;
      break;
    case I_ASSERT:
      if (assert_holds(in->x, prev, next)) stack[sp++] = pc + 1;
      break;
    case I_MATCH: matched = 1; break;
    case I_SET: L->pc[L->n++] = pc; break;
    }
  }
  return matched;
}

/* the code points of s[0, n) into cp (a byte that is not valid UTF-8 becomes 0x110000 + the byte, a
   value no set contains); returns their number */
static size_t code_points(const char *s, size_t n, int64_t *cp) {
  size_t m = 0;
  const unsigned char *u = (const unsigned char *)s;
  for (size_t i = 0; i < n;) {
    uint32_t c = u[i];
    int len = c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : (c & 0xF8) == 0xF0 ? 4 : 0;
    int ok = len > 0 && i + (size_t)len <= n;
    uint32_t v = len == 1 ? c : len == 2 ? (c & 0x1F) : len == 3 ? (c & 0x0F) : (c & 0x07);
    for (int k = 1; ok && k < len; ++k) {
      if ((u[i + (size_t)k] & 0xC0) != 0x80) ok = 0;
      else v = (v << 6) | (u[i + (size_t)k] & 0x3F);
    }
    if (ok && ((len == 2 && v < 0x80) || (len == 3 && v < 0x800) || (len == 4 && v < 0x10000) || v > 0x10FFFF ||
               (v >= 0xD800 && v <= 0xDFFF)))
      ok = 0;
    if (ok) {
      cp[m++] = v;
      i += (size_t)len;
    } else {
      cp[m++] = 0x110000 + c;
      i += 1;
    }
  }
  return m;
}

int orc_re_search(const orc_re *R, const char *s, size_t n) {
  int64_t small[256];
  int64_t *cp = n <= 256 ? small : (int64_t *)malloc(n * sizeof(int64_t));
  const size_t m = code_points(s, n, cp);
  const int nc = R->ncode;
  int *buf = (int *)malloc((size_t)nc * 2 * sizeof(int));
  uint32_t *mark = (uint32_t *)calloc((size_t)nc, sizeof(uint32_t));
  tlist cur = {buf, 0}, nxt = {buf + nc, 0};
  /* a closure pushes at most two targets per instruction it visits, plus its start */
  int *stack2 = (int *)malloc(((size_t)nc * 2 + 2) * sizeof(int));
  uint32_t g = 1; /* marks start at 0: generation 0 would read as visited */
  int found = 0;
  for (size_t i = 0; i <= m && !found; ++i) {
    int64_t prev = i ? cp[i - 1] : -1, next = i < m ? cp[i] : -1;
    /* threads carried from the previous step were added with this position's context already;
       a new thread starts here (unanchored search) */
    if (add_thread(R, &cur, mark, g, stack2, 0, prev, next)) found = 1;
    if (found || i == m) break;
    ++g;
    nxt.n = 0;
    int64_t after = i + 1 < m ? cp[i + 1] : -1;
    for (int t = 0; t < cur.n && !found; ++t) {
      const rinst *in = &R->code[cur.pc[t]];
      if (cs_has(&R->sets[in->x], (uint32_t)(cp[i] < 0x110000 ? cp[i] : 0xFFFFFFFFu)))
        if (add_thread(R, &nxt, mark, g, stack2, cur.pc[t] + 1, cp[i], after)) found = 1;
    }
    tlist tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  free(stack2);
  free(mark);
  free(buf);
  if (cp != small) free(cp);
  return found;
}

/* ------------------------------------------------------------------ globs
 * fnmatch(3) with flags 0 in a UTF-8 locale, restated over code points (the dialect DESIGN.md §2
 * fixes for the trusted-repos lists; the product compiles the same globs into its byte automata,
 * automaton.cpp parse_glob): `*` any string ('/' included, no leading-dot rule), `?` one character,
 * `[...]` one character of a set — `!` or `^` first negates, `]` first is literal, `a-z` ranges in
 * code point order, `[:name:]` the ASCII classes, `\` escapes — `\x` the character x. glibc rules
 * for the odd cases: an unterminated `[` is an ordinary character and a trailing `\` never matches.
 * Unlike libc fnmatch this does not depend on the process locale. */
typedef struct {
  int star;
  cset set;
} gtok;

/* the pattern's tokens; 0 = unsupported (not UTF-8, an unknown class, a collating element) */
static int glob_compile(const char *p, gtok **out, int *ntok, int *never) {
  size_t n = strlen(p);
  rparse P;
  memset(&P, 0, sizeof(P));
  P.p = p;
  P.n = n;
  for (P.at = 0; P.at < n;)
    if (next_char(&P) < 0) return 0;
  gtok *t = (gtok *)calloc(n + 1, sizeof(gtok));
  int k = 0;
  *never = 0;
  P.at = 0;
  while (P.at < n) {
    const int c = peek(&P);
    if (c == '*') {
      t[k++].star = 1;
      P.at++;
    } else if (c == '?') {
      cset none = {0};
      t[k++].set = cs_complement(&none);
      P.at++;
    } else if (c == '\\') {
      P.at++;
      if (at_end(&P)) {
        *never = 1;
        break;
      }
      int64_t x = next_char(&P);
      cs_push(&t[k++].set, (uint32_t)x, (uint32_t)x);
    } else if (c == '[') {
      size_t j = P.at + 1, save = P.at;
      int neg = 0, closed = 0, first = 1, bad_syntax = 0;
      cset s = {0};
      if (j < n && (p[j] == '!' || p[j] == '^')) neg = 1, j++;
      P.at = j;
      while (!at_end(&P)) {
        const int x = peek(&P);
        if (x == ']' && !first) {
          closed = 1;
          P.at++;
          break;
        }
        first = 0;
        if (x == '[' && P.at + 1 < n && p[P.at + 1] == ':') {
          /* a class name: letters a-y closed by ":]" (glibc), else '[' is a member */
          const char *e = p + P.at + 2;
          while (*e >= 'a' && *e < 'z') ++e;
          if (!(e[0] == ':' && e[1] == ']')) {
            cs_push(&s, '[', '[');
            P.at++;
            continue;
          }
          cset cl;
          const char *name = p + P.at + 2;
          const size_t len = (size_t)(e - name);
          /* the POSIX classes; [:ascii:] and [:word:] are regex-only names */
          if ((len == 5 && !memcmp(name, "ascii", 5)) || (len == 4 && !memcmp(name, "word", 4)) ||
              !named_class(name, len, &cl)) {
            bad_syntax = 1;
            break;
          }
          cs_add_all(&s, &cl);
          cs_free(&cl);
          P.at = (size_t)(e - p) + 2;
          continue;
        }
        if (x == '[' && P.at + 1 < n && (p[P.at + 1] == '.' || p[P.at + 1] == '=')) {
          bad_syntax = 1;
          break;
        }
        if (x == '\\') {
          if (P.at + 1 >= n) break; /* unterminated */
          P.at++;
        }
        const uint32_t lo = (uint32_t)next_char(&P);
        if (P.at < n && p[P.at] == '-' && (P.at + 1 == n || p[P.at + 1] != ']')) {
          P.at++;
          if (P.at < n && p[P.at] == '\\') P.at++;
          if (P.at == n) { /* the range has no upper end: glibc fails the match there */
            cs_free(&s);
            *never = 1;
            break;
          }
          const uint32_t hi = (uint32_t)next_char(&P);
          if (lo <= hi) cs_push(&s, lo, hi);
        } else {
          cs_push(&s, lo, lo);
        }
      }
      if (*never) break;
      if (bad_syntax) {
        cs_free(&s);
        for (int q = 0; q < k; ++q) cs_free(&t[q].set);
        free(t);
        return 0;
      }
      if (!closed) {
        cs_free(&s);
        cs_push(&t[k++].set, '[', '[');
        P.at = save + 1;
        continue;
      }
      cs_canon(&s);
      if (neg) {
        cset c2 = cs_complement(&s);
        cs_free(&s);
        s = c2;
      }
      t[k++].set = s;
    } else {
      int64_t x = next_char(&P);
      cs_push(&t[k++].set, (uint32_t)x, (uint32_t)x);
    }
  }
  *out = t;
  *ntok = k;
  return 1;
}

struct orc_glob {
  gtok *t;
  int n, never;
};

orc_glob *orc_glob_compile(const char *pattern) {
  orc_glob *g = (orc_glob *)calloc(1, sizeof(orc_glob));
  if (!glob_compile(pattern, &g->t, &g->n, &g->never)) {
    free(g);
    return NULL;
  }
  return g;
}

void orc_glob_free(orc_glob *g) {
  if (!g) return;
  for (int k = 0; k < g->n; ++k) cs_free(&g->t[k].set);
  free(g->t);
  free(g);
}

int orc_glob_run(const orc_glob *g, const char *s, size_t n) {
  if (g->never) return 0;
  const gtok *t = g->t;
  const int nt = g->n;
  int64_t small[256];
  int64_t *cp = n <= 256 ? small : (int64_t *)malloc(n * sizeof(int64_t));
  const size_t m = code_points(s, n, cp);
  /* one `*` restart point suffices: the tokens between stars match one character each */
  int i = 0, star = -1, found = 0;
  size_t j = 0, star_j = 0;
  for (;;) {
    if (j < m && i < nt && !t[i].star && cs_has(&t[i].set, (uint32_t)cp[j])) {
      i++, j++;
    } else if (i < nt && t[i].star) {
      star = i++;
      star_j = j;
    } else if (j == m && i == nt) {
      found = 1;
      break;
    } else if (star >= 0 && star_j < m) {
      i = star + 1;
      j = ++star_j;
    } else {
      break;
    }
  }
  if (cp != small) free(cp);
  return found;
}

int orc_glob_ok(const char *pattern) {
  orc_glob *g = orc_glob_compile(pattern);
  orc_glob_free(g);
  return g != NULL;
}

int orc_glob_match(const char *pattern, const char *s, size_t n) {
  orc_glob *g = orc_glob_compile(pattern);
  if (!g) return -1;
  const int r = orc_glob_run(g, s, n);
  orc_glob_free(g);
  return r;
}
