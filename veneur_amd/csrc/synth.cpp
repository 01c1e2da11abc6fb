// synth.cpp -- deterministic synthetic DogStatsD-shaped streams (see veneur_amd_synth.h).
#include "../../include/veneur_amd_synth.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
inline double u01(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

uint32_t fnv1a(const char* s, size_t n, uint32_t h) {
  for (size_t i = 0; i < n; i++) {
    h ^= (uint8_t)s[i];
    h *= 16777619u;
  }
  return h;
}

const char* kTypeName[4] = {"counter", "gauge", "histogram", "set"};

struct Part {
  std::vector<uint32_t> slot[4];
  std::vector<double> val[3];
  std::vector<float> rate[3];
  std::vector<uint32_t> mlen;
  std::vector<uint8_t> mbytes;
};

template <class T>
T* copy_out(const std::vector<std::vector<T>*>& parts) {
  size_t n = 0;
  for (auto* p : parts) n += p->size();
  T* out = (T*)malloc(std::max<size_t>(n, 1) * sizeof(T));
  size_t o = 0;
  for (auto* p : parts) {
    if (!p->empty()) memcpy(out + o, p->data(), p->size() * sizeof(T));
    o += p->size();
  }
  return out;
}

}  // namespace

extern "C" int vn_synth_generate(const vn_synth_config* cfg, vn_synth_out* out) {
  if (!cfg || !out || cfg->n_keys == 0 || cfg->n_shards == 0) return -1;
  memset(out, 0, sizeof(*out));
  const uint32_t K = cfg->n_keys;
  // ---- key table: class, digest, shard membership
  std::vector<int8_t> cls(K);
  std::vector<uint32_t> dig(K), kslot(K, 0xffffffffu);
  double cum[4];
  double tot = cfg->mix[0] + cfg->mix[1] + cfg->mix[2] + cfg->mix[3];
  double run = 0;
  for (int c = 0; c < 4; c++) {
    run += cfg->mix[c] / tot;
    cum[c] = run;
  }
  std::vector<uint32_t> shard_keys;
  std::vector<uint32_t> key_of[4], dig_of[4];
  char name[32];
  for (uint32_t k = 0; k < K; k++) {
    double u = u01(splitmix64(cfg->seed ^ (0xA5A5A5A5ull + (uint64_t)k * 0x9E3779B97F4A7C15ull)));
    int c = 0;
    while (c < 3 && u >= cum[c]) c++;
    while (c < 3 && cfg->mix[c] == 0) c++;
    cls[k] = (int8_t)c;
    int n = snprintf(name, sizeof(name), "k%07u", k);
    uint32_t h = fnv1a(name, (size_t)n, 2166136261u);
    h = fnv1a(kTypeName[c], strlen(kTypeName[c]), h);
    dig[k] = h;
    if (h % cfg->n_shards == cfg->shard) {
      shard_keys.push_back(k);
      kslot[k] = (uint32_t)key_of[c].size();
      key_of[c].push_back(k);
      dig_of[c].push_back(h);
    }
  }
  if (shard_keys.empty()) return -2;
  // ---- Zipf CDF over the shard's keys (key id = global popularity rank)
  std::vector<double> cdf(shard_keys.size());
  double acc = 0;
  for (size_t i = 0; i < shard_keys.size(); i++) {
    acc += cfg->zipf_s == 0 ? 1.0 : 1.0 / std::pow((double)shard_keys[i] + 1.0, cfg->zipf_s);
    cdf[i] = acc;
  }
  for (auto& v : cdf) v /= acc;
  cdf.back() = 1.0;

  int T = cfg->threads > 0 ? cfg->threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  const uint64_t N = cfg->n_samples;
  std::vector<Part> parts((size_t)T);
  auto work = [&](int t) {
    Part& P = parts[(size_t)t];
    uint64_t lo = N * (uint64_t)t / (uint64_t)T, hi = N * (uint64_t)(t + 1) / (uint64_t)T;
    char mb[32];
    for (uint64_t i = lo; i < hi; i++) {
      uint64_t r0 = splitmix64(cfg->seed * 0x100000001B3ull + i);
      uint64_t r1 = splitmix64(r0), r2 = splitmix64(r1), r3 = splitmix64(r2);
      double u = u01(r0);
      size_t ki = (size_t)(std::upper_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
      if (ki >= cdf.size()) ki = cdf.size() - 1;
      uint32_t key = shard_keys[ki];
      int c = cls[key];
      uint32_t s = kslot[key];
      double ur = u01(r2);
      float rate = ur < cfg->rate_tenth ? 0.1f : (ur < cfg->rate_tenth + cfg->rate_half ? 0.5f : 1.0f);
      P.slot[c].push_back(s);
      if (c == 0) {  // counter: uniform int 1..10
        P.val[0].push_back((double)(1 + (r1 % 10)));
        P.rate[0].push_back(rate);
      } else if (c == 1) {  // gauge: uniform(0, 1000)
        P.val[1].push_back(u01(r1) * 1000.0);
      } else if (c == 2) {  // timer: lognormal(mu, sigma) via Box-Muller
        double a = u01(r1), b = u01(r3);
        if (a < 1e-300) a = 1e-300;
        double z = std::sqrt(-2.0 * std::log(a)) * std::cos(6.283185307179586 * b);
        P.val[2].push_back(std::exp(cfg->histo_mu + cfg->histo_sigma * z));
        P.rate[2].push_back(rate);
      } else {  // set member "m%010llu"
        unsigned long long m = cfg->member_universe ? (r1 % cfg->member_universe) : r1;
        int n = snprintf(mb, sizeof(mb), "m%010llu", m);
        P.mlen.push_back((uint32_t)n);
        P.mbytes.insert(P.mbytes.end(), mb, mb + n);
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) th.emplace_back(work, t);
  for (auto& x : th) x.join();

  for (int c = 0; c < 4; c++) {
    out->n_slots[c] = (uint32_t)key_of[c].size();
    out->key_of_slot[c] = (uint32_t*)malloc(std::max<size_t>(1, key_of[c].size()) * 4);
    out->digest_of_slot[c] = (uint32_t*)malloc(std::max<size_t>(1, key_of[c].size()) * 4);
    if (!key_of[c].empty()) {
      memcpy(out->key_of_slot[c], key_of[c].data(), key_of[c].size() * 4);
      memcpy(out->digest_of_slot[c], dig_of[c].data(), dig_of[c].size() * 4);
    }
    std::vector<std::vector<uint32_t>*> sp;
    for (auto& P : parts) sp.push_back(&P.slot[c]);
    uint32_t* sl = copy_out(sp);
    out->n[c] = 0;
    for (auto* p : sp) out->n[c] += p->size();
    if (c == 0) out->c_slot = sl;
    if (c == 1) out->g_slot = sl;
    if (c == 2) out->h_slot = sl;
    if (c == 3) out->s_slot = sl;
  }
  for (int c = 0; c < 3; c++) {
    std::vector<std::vector<double>*> vp;
    std::vector<std::vector<float>*> rp;
    for (auto& P : parts) {
      vp.push_back(&P.val[c]);
      rp.push_back(&P.rate[c]);
    }
    double* v = copy_out(vp);
    float* r = copy_out(rp);
    if (c == 0) { out->c_val = v; out->c_rate = r; }
    if (c == 1) { out->g_val = v; free(r); }
    if (c == 2) { out->h_val = v; out->h_rate = r; }
  }
  // set member offsets and bytes
  uint64_t ns = out->n[3], nb = 0;
  for (auto& P : parts) nb += P.mbytes.size();
  out->s_off = (uint32_t*)malloc((ns + 1) * 4);
  out->s_bytes = (uint8_t*)malloc(std::max<uint64_t>(nb, 1));
  out->s_nbytes = nb;
  uint64_t o = 0, j = 0;
  for (auto& P : parts) {
    for (uint32_t l : P.mlen) {
      out->s_off[j++] = (uint32_t)o;
      o += l;
    }
  }
  out->s_off[ns] = (uint32_t)o;
  o = 0;
  for (auto& P : parts) {
    if (!P.mbytes.empty()) memcpy(out->s_bytes + o, P.mbytes.data(), P.mbytes.size());
    o += P.mbytes.size();
  }
  return 0;
}

extern "C" void vn_synth_free(vn_synth_out* o) {
  if (!o) return;
  free(o->c_slot); free(o->c_val); free(o->c_rate);
  free(o->g_slot); free(o->g_val);
  free(o->h_slot); free(o->h_val); free(o->h_rate);
  free(o->s_slot); free(o->s_off); free(o->s_bytes);
  for (int c = 0; c < 4; c++) {
    free(o->key_of_slot[c]);
    free(o->digest_of_slot[c]);
  }
  memset(o, 0, sizeof(*o));
}
