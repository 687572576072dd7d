// synth.cpp — libkwsynth.so: seeded synthetic AdmissionReview workloads.
// Bench / test infrastructure, not part of the product library. Produces the kw_soa columns of a
// batch directly (fast, for 1M-10M rows) and, for any row, the AdmissionReview JSON document that
// flattens to exactly those columns (the flattener parity test checks this).
//
// Distribution: uid UUIDv4; operation CREATE 80 % / UPDATE 20 %; namespace
// Zipf(1.1) over ns-000..ns-255 plus special namespaces; containers 1+Geom(0.5) capped at 16
// (config 5: Zipf(1.3) over 1..64); image registry in {none 25 %, docker.io, ghcr.io, quay.io,
// registry.k8s.io, gcr.io, my-corp.example:5000}, 1-3 path segments, tag in {absent 20 %, latest
// 15 %, semver 50 %, digest 15 %}; labels Poisson(4) from a 24-key vocabulary; AppArmor annotation
// on 30 % of containers; capabilities.add Poisson(0.5) from 14 names, drop ["ALL"] 50 %;
// privileged 5 %; config 5 mixes Pod 70 % / Deployment 20 % / Namespace 10 %.
// Config 6 (configs/c6_256.yml) draws from that config's larger vocabularies: registries
// reg-000..239.example.com (60 %) with paths team-NN/..., 150 extra label keys, AppArmor profiles
// localhost/prof-00..99, namespaces ns-000..255 uniform.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kwgpu.h"

namespace {

struct Rng {
  uint64_t s[4];
  static uint64_t sm(uint64_t& x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  explicit Rng(uint64_t seed) {
    for (auto& v : s) v = sm(seed);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {  // xoshiro256**
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(uni() * n); }
  bool chance(double p) { return uni() < p; }
  uint32_t poisson(double lam) {
    double L = std::exp(-lam), p = 1;
    uint32_t k = 0;
    do {
      ++k;
      p *= uni();
    } while (p > L);
    return k - 1;
  }
};

struct Zipf {
  std::vector<double> cdf;
  Zipf(int n, double s) {
    double acc = 0;
    for (int k = 1; k <= n; ++k) {
      acc += 1.0 / std::pow((double)k, s);
      cdf.push_back(acc);
    }
    for (auto& c : cdf) c /= acc;
  }
  int draw(Rng& r) const { return (int)(std::lower_bound(cdf.begin(), cdf.end(), r.uni()) - cdf.begin()); }
};

const char* kRegistries[] = {"docker.io", "ghcr.io", "quay.io", "registry.k8s.io", "gcr.io", "my-corp.example:5000"};
const char* kCaps[] = {"NET_ADMIN", "SYS_TIME", "SYS_ADMIN", "NET_RAW", "CHOWN", "KILL", "SETUID",
                       "SETGID", "DAC_OVERRIDE", "FOWNER", "MKNOD", "AUDIT_WRITE", "SYS_PTRACE", "NET_BIND_SERVICE"};
const char* kLabelKeys[] = {"app", "tier", "env", "team", "owner", "version", "release", "component",
                            "part-of", "managed-by", "app.kubernetes.io/name", "app.kubernetes.io/instance",
                            "app.kubernetes.io/version", "app.kubernetes.io/component", "app.kubernetes.io/part-of",
                            "app.kubernetes.io/managed-by", "cost-center", "region", "zone", "critical", "debug",
                            "experimental", "legacy", "pci"};
const char* kLabelValues[] = {"frontend", "backend", "db", "cache", "dev", "staging", "prod", "team-a", "team-blue",
                              "v1.2.3", "v2.0", "true", "false", "eu-west-1", "us-east-2", "1234", "payments", "web",
                              "x", "Not_Valid!"};
const char* kHex = "0123456789abcdef";

struct StrCol {
  std::vector<uint32_t> off{0};
  std::vector<uint8_t> bytes;
  void push(const std::string& s) {
    bytes.insert(bytes.end(), s.begin(), s.end());
    off.push_back((uint32_t)bytes.size());
  }
  kw_strcol view() const { return kw_strcol{off.data(), bytes.data(), off.size() - 1}; }
  std::string at(size_t i) const { return std::string((const char*)bytes.data() + off[i], off[i + 1] - off[i]); }
  void append(const StrCol& o) {
    const uint32_t base = off.back();
    bytes.insert(bytes.end(), o.bytes.begin(), o.bytes.end());
    for (size_t i = 1; i < o.off.size(); ++i) off.push_back(base + o.off[i]);
  }
};

}  // namespace

struct kws_batch {
  int config = 0;
  uint64_t n = 0;
  std::vector<uint8_t> req_flags, ctr_flags, obj_kind;  // obj_kind: 0 Pod, 1 Deployment, 2 Namespace
  std::vector<uint32_t> ctr_off{0}, lbl_off{0}, capadd_off{0}, capdrop_off{0};
  StrCol uid, ns, op, kind, name, ctr_name, ctr_image, ctr_aa, cap_add, cap_drop, lbl_key, lbl_val;
};

namespace {

std::string rand_word(Rng& r, int lo, int hi) {
  static const char* al = "abcdefghijklmnopqrstuvwxyz0123456789-";
  int n = lo + (int)r.below((uint32_t)(hi - lo + 1));
  std::string s;
  for (int i = 0; i < n; ++i) s.push_back(al[r.below(i == 0 || i == n - 1 ? 36 : 37)]);
  return s;
}

std::string image(Rng& r, int config) {
  std::string s;
  int segs = 1 + (int)r.below(3);
  if (config == 6 && r.chance(0.6)) {
    char buf[64];
    const uint32_t k = r.below(240);
    snprintf(buf, sizeof(buf), "reg-%03u.example.com/team-%02u/", k, r.chance(0.7) ? k % 40 : r.below(40));
    s = buf;
    segs = 1;
  } else if (!r.chance(0.25)) {
    s = kRegistries[r.below(6)];
    s += "/";
  }
  for (int i = 0; i < segs; ++i) {
    if (i) s += "/";
    s += rand_word(r, 3, 12);
  }
  double t = r.uni();
  if (t < 0.20) {
  } else if (t < 0.35) {
    s += ":latest";
  } else if (t < 0.85) {
    s += ":" + std::to_string(r.below(5)) + "." + std::to_string(r.below(20)) + "." + std::to_string(r.below(10));
  } else {
    s += "@sha256:";
    for (int i = 0; i < 64; ++i) s.push_back(kHex[r.below(16)]);
  }
  return s;
}

std::string uuid4(Rng& r) {
  std::string s;
  for (int i = 0; i < 36; ++i) {
    if (i == 8 || i == 13 || i == 18 || i == 23) s.push_back('-');
    else if (i == 14) s.push_back('4');
    else if (i == 19) s.push_back(kHex[8 + r.below(4)]);
    else s.push_back(kHex[r.below(16)]);
  }
  return s;
}

void json_str(std::string* o, const std::string& s) {
  o->push_back('"');
  for (char c : s) {
    if (c == '"' || c == '\\') o->push_back('\\');
    o->push_back(c);
  }
  o->push_back('"');
}

}  // namespace

namespace {
kws_batch* generate_range(int config, uint64_t n, uint64_t seed, uint64_t row0);

// The shape of a row, drawn from its own generator so that it can be computed without generating
// the row (kws_shard_bounds balances shards by it): the object kind and the container counts.
struct Shape {
  int ok = 0;  // 0 Pod, 1 Deployment, 2 Namespace
  uint32_t nc = 0, ninit = 0, neph = 0;
  uint32_t containers() const { return nc + ninit + neph; }
};

Shape row_shape(int config, uint64_t seed, uint64_t row) {
  static const Zipf zc5(64, 1.3);
  Rng r(seed * 0x9e3779b97f4a7c15ull + row * 0x100000001b3ull + 777);
  Shape sh;
  if (config == 5 || config == 0) {
    const double u = r.uni();
    sh.ok = u < 0.70 ? 0 : u < 0.90 ? 1 : 2;
  }
  if (sh.ok == 2) return sh;
  if (config == 5) {
    sh.nc = 1 + (uint32_t)zc5.draw(r);
  } else {
    sh.nc = 1;
    while (sh.nc < 16 && r.chance(0.5)) ++sh.nc;
  }
  sh.ninit = (config == 0 || config == 5) && r.chance(0.1) ? 1 : 0;
  sh.neph = config == 0 && r.chance(0.03) ? 1 : 0;
  return sh;
}

void append_batch(kws_batch* d, const kws_batch& o) {
  auto shift = [](std::vector<uint32_t>* dst, const std::vector<uint32_t>& src) {
    const uint32_t base = dst->back();
    for (size_t i = 1; i < src.size(); ++i) dst->push_back(base + src[i]);
  };
  d->n += o.n;
  d->req_flags.insert(d->req_flags.end(), o.req_flags.begin(), o.req_flags.end());
  d->ctr_flags.insert(d->ctr_flags.end(), o.ctr_flags.begin(), o.ctr_flags.end());
  d->obj_kind.insert(d->obj_kind.end(), o.obj_kind.begin(), o.obj_kind.end());
  shift(&d->ctr_off, o.ctr_off);
  shift(&d->lbl_off, o.lbl_off);
  shift(&d->capadd_off, o.capadd_off);
  shift(&d->capdrop_off, o.capdrop_off);
  StrCol* mine[] = {&d->uid, &d->ns, &d->op, &d->kind, &d->name, &d->ctr_name, &d->ctr_image, &d->ctr_aa,
                    &d->cap_add, &d->cap_drop, &d->lbl_key, &d->lbl_val};
  const StrCol* theirs[] = {&o.uid, &o.ns, &o.op, &o.kind, &o.name, &o.ctr_name, &o.ctr_image, &o.ctr_aa,
                            &o.cap_add, &o.cap_drop, &o.lbl_key, &o.lbl_val};
  for (size_t k = 0; k < sizeof(mine) / sizeof(mine[0]); ++k) mine[k]->append(*theirs[k]);
}
}  // namespace

extern "C" {

// config: 1..6 as in SURVEY §8(d) (1: namespace-heavy, 5: mixed kinds + skewed containers, 6: the
// c6_256 vocabularies); 0 = parity mix (all kinds, every field exercised). Rows [row0, row0+n) of
// the seeded stream (every row has its own generator, so large batches are made on 16 threads).
kws_batch* kws_generate(int config, uint64_t n, uint64_t seed, uint64_t row0) {
  const uint64_t nt = n >= 200000 ? 16 : 1;
  if (nt == 1) return generate_range(config, n, seed, row0);
  std::vector<kws_batch*> part(nt);
  std::vector<std::thread> th;
  for (uint64_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] { part[t] = generate_range(config, n * (t + 1) / nt - n * t / nt, seed, row0 + n * t / nt); });
  for (auto& x : th) x.join();
  kws_batch* b = part[0];
  for (uint64_t t = 1; t < nt; ++t) {
    append_batch(b, *part[t]);
    delete part[t];
  }
  b->config = config;
  return b;
}

// Row weights of the synthetic stream: weight(row) = 1 + its containers (the per-request and
// per-container work of a pass). Splits rows [0, total) into `world` contiguous shards of equal
// weight: bounds[0] = 0 <= bounds[1] <= ... <= bounds[world] = total (C5's Zipf
// container counts make equal row counts unequal work). Computed on 16 threads from the row shapes
// alone, so every rank derives the same bounds without generating the other shards.
int kws_shard_bounds(int config, uint64_t total, uint64_t seed, int world, uint64_t* bounds) {
  if (world < 1 || !bounds) return 1;
  const uint64_t nt = total >= 200000 ? 16 : 1;
  std::vector<uint64_t> csum(nt + 1, 0);
  auto w = [&](uint64_t row) { return (uint64_t)1 + row_shape(config, seed, row).containers(); };
  {
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        uint64_t acc = 0;
        for (uint64_t r = total * t / nt; r < total * (t + 1) / nt; ++r) acc += w(r);
        csum[t + 1] = acc;
      });
    for (auto& x : th) x.join();
  }
  for (uint64_t t = 0; t < nt; ++t) csum[t + 1] += csum[t];
  const uint64_t W = csum[nt];
  bounds[0] = 0;
  bounds[world] = total;
  for (int k = 1; k < world; ++k) {
    const unsigned __int128 tgt128 = (unsigned __int128)W * (uint64_t)k / (uint64_t)world;
    const uint64_t target = (uint64_t)tgt128;  // shard k starts at the first row whose prefix reaches it
    uint64_t t = 0;
    while (t + 1 < nt && csum[t + 1] <= target) ++t;
    uint64_t acc = csum[t], r = total * t / nt;
    const uint64_t end = total * (t + 1) / nt;
    while (r < end && acc + w(r) <= target) acc += w(r++);
    if (acc < target && r < end) ++r;  // the row straddling the target goes to the earlier shard
    bounds[k] = std::max(bounds[k - 1], r);
  }
  return 0;
}

// Containers per row for rows [row0, row0 + n) (tests check the bounds against these).
int kws_row_containers(int config, uint64_t n, uint64_t seed, uint64_t row0, uint32_t* out) {
  for (uint64_t i = 0; i < n; ++i) out[i] = row_shape(config, seed, row0 + i).containers();
  return 0;
}

}  // extern "C"

namespace {
kws_batch* generate_range(int config, uint64_t n, uint64_t seed, uint64_t row0) {
  auto* b = new kws_batch();
  b->config = config;
  b->n = n;
  static const Zipf zns(256, 1.1);
  b->req_flags.reserve(n);
  for (uint64_t i = 0; i < n; ++i) {
    Rng r(seed * 0x100000001b3ull + (row0 + i) * 0x9e3779b97f4a7c15ull + 12345);
    const Shape sh = row_shape(config, seed, row0 + i);
    const int ok = sh.ok;  // kind of object
    b->obj_kind.push_back((uint8_t)ok);
    uint8_t rf = KW_REQ_HAS_OBJECT;
    b->uid.push(uuid4(r));
    b->op.push(r.chance(0.8) ? "CREATE" : "UPDATE");
    b->kind.push(ok == 0 ? "Pod" : ok == 1 ? "Deployment" : "Namespace");
    std::string nsn;
    double sp = r.uni();
    if (config == 1 && sp < 0.5) nsn = "kubewarden-approved";
    else if (config != 1 && sp < 0.03) nsn = "kubewarden";
    else if (config == 0 && sp < 0.05) nsn = "kubewarden-approved";
    else if (config == 6) {
      char buf[16];
      snprintf(buf, sizeof(buf), "ns-%03u", r.below(256));
      nsn = buf;
    } else {
      char buf[16];
      snprintf(buf, sizeof(buf), "ns-%03d", zns.draw(r));
      nsn = buf;
    }
    bool has_ns = ok != 2 || config == 0 ? !(config == 0 && r.chance(0.02)) : false;
    if (has_ns) rf |= KW_REQ_HAS_NAMESPACE;
    b->ns.push(has_ns ? nsn : "");
    b->name.push(rand_word(r, 4, 16));
    // labels of the object
    uint32_t nl = std::min<uint32_t>(r.poisson(4.0), 20);
    std::vector<int> used;
    for (uint32_t k = 0; k < nl; ++k) {
      int key = (int)r.below(config == 6 ? 174 : 24);
      if (std::find(used.begin(), used.end(), key) != used.end()) continue;
      used.push_back(key);
      if (key < 24) {
        b->lbl_key.push(kLabelKeys[key]);
      } else {
        char buf[32];
        snprintf(buf, sizeof(buf), "team.example/k-%03d", key - 24);
        b->lbl_key.push(buf);
      }
      b->lbl_val.push(r.chance(0.15) ? rand_word(r, 1, 20) : kLabelValues[r.below(20)]);
    }
    b->lbl_off.push_back((uint32_t)b->lbl_key.off.size() - 1);
    // containers
    if (ok != 2) {
      rf |= KW_REQ_HAS_PODSPEC;
      const uint32_t nc = sh.nc, ninit = sh.ninit, neph = sh.neph;
      std::vector<std::string> names;
      for (uint32_t c = 0; c < nc + ninit + neph; ++c) {
        uint8_t cf = KW_CTR_HAS_IMAGE;
        if (c >= nc) cf |= c < nc + ninit ? KW_CTR_INIT : KW_CTR_EPHEMERAL;
        std::string cname = "c" + std::to_string(c) + "-" + rand_word(r, 3, 8);
        b->ctr_name.push(cname);
        b->ctr_image.push(image(r, config));
        if (r.chance(0.05)) cf |= KW_CTR_PRIVILEGED;
        uint32_t na = std::min<uint32_t>(r.poisson(0.5), 6);
        for (uint32_t k = 0; k < na; ++k) b->cap_add.push(kCaps[r.below(14)]);
        b->capadd_off.push_back((uint32_t)b->cap_add.off.size() - 1);
        if (r.chance(0.5)) b->cap_drop.push("ALL");
        else {
          uint32_t nd = r.below(3);
          for (uint32_t k = 0; k < nd; ++k) b->cap_drop.push(kCaps[r.below(14)]);
        }
        b->capdrop_off.push_back((uint32_t)b->cap_drop.off.size() - 1);
        if (r.chance(0.3)) {
          cf |= KW_CTR_HAS_APPARMOR;
          double u = r.uni();
          if (config == 6) {
            char buf[32];
            snprintf(buf, sizeof(buf), "localhost/prof-%02u", r.below(100));
            b->ctr_aa.push(u < 0.3 ? std::string("runtime/default") : std::string(buf));
          } else {
            b->ctr_aa.push(u < 0.5 ? "runtime/default" : u < 0.85 ? "localhost/p" + std::to_string(r.below(10)) : "unconfined");
          }
        } else {
          b->ctr_aa.push("");
        }
        b->ctr_flags.push_back(cf);
      }
    }
    b->ctr_off.push_back((uint32_t)b->ctr_flags.size());
    b->req_flags.push_back(rf);
  }
  return b;
}
}  // namespace

extern "C" {

void kws_free(kws_batch* b) { delete b; }

int kws_view(const kws_batch* b, kw_soa* s) {
  memset(s, 0, sizeof(*s));
  s->n_requests = b->n;
  s->req_flags = b->req_flags.data();
  s->ctr_off = b->ctr_off.data();
  s->lbl_off = b->lbl_off.data();
  s->uid = b->uid.view();
  s->ns = b->ns.view();
  s->op = b->op.view();
  s->kind = b->kind.view();
  s->ctr_flags = b->ctr_flags.data();
  s->capadd_off = b->capadd_off.data();
  s->capdrop_off = b->capdrop_off.data();
  s->ctr_name = b->ctr_name.view();
  s->ctr_image = b->ctr_image.view();
  s->ctr_apparmor = b->ctr_aa.view();
  s->cap_add = b->cap_add.view();
  s->cap_drop = b->cap_drop.view();
  s->lbl_key = b->lbl_key.view();
  s->lbl_val = b->lbl_val.view();
  return 0;
}

// AdmissionReview JSON of one row (flattens to exactly this row's columns).
int kws_json(const kws_batch* b, uint64_t row, char* buf, size_t cap, size_t* need) {
  std::string o;
  int ok = b->obj_kind[row];
  const char* kind = ok == 0 ? "Pod" : ok == 1 ? "Deployment" : "Namespace";
  const char* group = ok == 1 ? "apps" : "";
  const char* res = ok == 0 ? "pods" : ok == 1 ? "deployments" : "namespaces";
  bool has_ns = b->req_flags[row] & KW_REQ_HAS_NAMESPACE;
  o += "{\"apiVersion\":\"admission.k8s.io/v1\",\"kind\":\"AdmissionReview\",\"request\":{\"uid\":";
  json_str(&o, b->uid.at(row));
  o += std::string(",\"kind\":{\"group\":\"") + group + "\",\"version\":\"v1\",\"kind\":\"" + kind + "\"}";
  o += std::string(",\"resource\":{\"group\":\"") + group + "\",\"version\":\"v1\",\"resource\":\"" + res + "\"}";
  o += ",\"name\":";
  json_str(&o, b->name.at(row));
  if (has_ns) {
    o += ",\"namespace\":";
    json_str(&o, b->ns.at(row));
  }
  o += ",\"operation\":";
  json_str(&o, b->op.at(row));
  o += ",\"userInfo\":{\"username\":\"kubernetes-admin\",\"groups\":[\"system:masters\",\"system:authenticated\"]}";
  o += std::string(",\"object\":{\"apiVersion\":\"") + (ok == 1 ? "apps/v1" : "v1") + "\",\"kind\":\"" + kind + "\"";
  o += ",\"metadata\":{\"name\":";
  json_str(&o, b->name.at(row));
  if (has_ns) {
    o += ",\"namespace\":";
    json_str(&o, b->ns.at(row));
  }
  o += ",\"labels\":{";
  for (uint32_t l = b->lbl_off[row]; l < b->lbl_off[row + 1]; ++l) {
    if (l != b->lbl_off[row]) o += ",";
    json_str(&o, b->lbl_key.at(l));
    o += ":";
    json_str(&o, b->lbl_val.at(l));
  }
  o += "}";
  uint32_t cb = b->ctr_off[row], ce = b->ctr_off[row + 1];
  auto annotations = [&]() {
    std::string a = "\"annotations\":{\"kubectl.kubernetes.io/last-applied-configuration\":\"{}\"";
    for (uint32_t c = cb; c < ce; ++c)
      if (b->ctr_flags[c] & KW_CTR_HAS_APPARMOR) {
        a += ",";
        json_str(&a, "container.apparmor.security.beta.kubernetes.io/" + b->ctr_name.at(c));
        a += ":";
        json_str(&a, b->ctr_aa.at(c));
      }
    return a + "}";
  };
  auto podspec = [&]() {
    std::string s = "{";
    const char* lists[3] = {"containers", "initContainers", "ephemeralContainers"};
    const uint8_t kinds[3] = {0, KW_CTR_INIT, KW_CTR_EPHEMERAL};
    bool first_list = true;
    for (int li = 0; li < 3; ++li) {
      std::string items;
      for (uint32_t c = cb; c < ce; ++c) {
        if ((b->ctr_flags[c] & (KW_CTR_INIT | KW_CTR_EPHEMERAL)) != kinds[li]) continue;
        if (!items.empty()) items += ",";
        items += "{\"name\":";
        json_str(&items, b->ctr_name.at(c));
        items += ",\"image\":";
        json_str(&items, b->ctr_image.at(c));
        items += ",\"imagePullPolicy\":\"IfNotPresent\",\"securityContext\":{";
        items += (b->ctr_flags[c] & KW_CTR_PRIVILEGED) ? "\"privileged\":true" : "\"privileged\":false";
        items += ",\"capabilities\":{\"add\":[";
        for (uint32_t k = b->capadd_off[c]; k < b->capadd_off[c + 1]; ++k) {
          if (k != b->capadd_off[c]) items += ",";
          json_str(&items, b->cap_add.at(k));
        }
        items += "],\"drop\":[";
        for (uint32_t k = b->capdrop_off[c]; k < b->capdrop_off[c + 1]; ++k) {
          if (k != b->capdrop_off[c]) items += ",";
          json_str(&items, b->cap_drop.at(k));
        }
        items += "]}}}";
      }
      if (items.empty() && li > 0) continue;
      if (!first_list) s += ",";
      first_list = false;
      s += std::string("\"") + lists[li] + "\":[" + items + "]";
    }
    return s + ",\"restartPolicy\":\"Always\",\"dnsPolicy\":\"ClusterFirst\"}";
  };
  if (ok == 0) {
    o += "," + annotations() + "}";
    o += ",\"spec\":" + podspec();
  } else if (ok == 1) {
    o += "}";
    o += ",\"spec\":{\"replicas\":3,\"template\":{\"metadata\":{" + annotations() + "},\"spec\":" + podspec() + "}}";
  } else {
    o += "}";
  }
  o += "},\"oldObject\":null,\"dryRun\":false,\"options\":{\"kind\":\"CreateOptions\",\"apiVersion\":\"meta.k8s.io/v1\"}}}";
  if (need) *need = o.size() + 1;
  if (!buf || cap < o.size() + 1) return 19;
  memcpy(buf, o.data(), o.size() + 1);
  return 0;
}

}  // extern "C"
