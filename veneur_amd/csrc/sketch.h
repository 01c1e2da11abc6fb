// sketch.h -- device/host primitives of the HLL member path.
//
//   metro64      vendor/github.com/dgryski/go-metro/metro64.go:7-85 (== metro_amd64.s), seed 1337
//                (vendor/github.com/axiomhq/hyperloglog/utils.go:66-70)
//   clz          vendor/github.com/dgryski/go-bits/clz_amd64.s (BSR; Clz(0) = 64)
//   encode_hash  vendor/github.com/axiomhq/hyperloglog/sparse.go:14-22  (p=14, pp=25)
//   decode_hash  sparse.go:25-35 + getIndex 7-12; decode(encode(x)) == getPosVal(x) (utils.go:46-51)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gomath.h"

namespace vn {

constexpr uint32_t kHllP = 14;
constexpr uint32_t kHllPP = 25;
constexpr uint32_t kHllM = 1u << kHllP;            // 16384 registers
constexpr uint32_t kHllMP = 1u << kHllPP;          // 2^25
constexpr uint32_t kHllCapacity = 16;              // 4-bit registers with base b
constexpr uint32_t kHllTmpTrigger = 164;           // len(tmpSet)*100 > m  <=>  len >= 164
constexpr uint32_t kHllListCap = 16640;            // >= 16384 + 164 codes (1 byte min per code)
constexpr uint32_t kHllNoCode = 0xffffffffu;       // never a valid sparse code
constexpr uint64_t kMetroSeed = 1337;

VN_HD uint64_t clz64(uint64_t x) { return x == 0 ? 64 : (uint64_t)__builtin_clzll(x); }
VN_HD uint64_t rotr64(uint64_t v, unsigned k) { return (v >> k) | (v << (64 - k)); }

template <class Load8, class Load4, class Load2, class Load1>
VN_HD uint64_t metro64_impl(uint32_t len, uint64_t seed, Load8 l8, Load4 l4, Load2 l2, Load1 l1) {
  const uint64_t k0 = 0xD6D018F5ull, k1 = 0xA2AA033Bull, k2 = 0x62992FC1ull, k3 = 0x30BC5B29ull;
  uint32_t p = 0;
  uint64_t hash = (seed + k2) * k0;
  if (len >= 32) {
    uint64_t v0 = hash, v1 = hash, v2 = hash, v3 = hash;
    while (len - p >= 32) {
      v0 += l8(p) * k0; v0 = rotr64(v0, 29) + v2;
      v1 += l8(p + 8) * k1; v1 = rotr64(v1, 29) + v3;
      v2 += l8(p + 16) * k2; v2 = rotr64(v2, 29) + v0;
      v3 += l8(p + 24) * k3; v3 = rotr64(v3, 29) + v1;
      p += 32;
    }
    v2 ^= rotr64(((v0 + v3) * k0) + v1, 37) * k1;
    v3 ^= rotr64(((v1 + v2) * k1) + v0, 37) * k0;
    v0 ^= rotr64(((v0 + v2) * k0) + v3, 37) * k1;
    v1 ^= rotr64(((v1 + v3) * k1) + v2, 37) * k0;
    hash += v0 ^ v1;
  }
  if (len - p >= 16) {
    uint64_t v0 = hash + (l8(p) * k2); v0 = rotr64(v0, 29) * k3;
    uint64_t v1 = hash + (l8(p + 8) * k2); v1 = rotr64(v1, 29) * k3;
    v0 ^= rotr64(v0 * k0, 21) + v1;
    v1 ^= rotr64(v1 * k3, 21) + v0;
    hash += v1;
    p += 16;
  }
  if (len - p >= 8) { hash += l8(p) * k3; p += 8; hash ^= rotr64(hash, 55) * k1; }
  if (len - p >= 4) { hash += (uint64_t)l4(p) * k3; p += 4; hash ^= rotr64(hash, 26) * k1; }
  if (len - p >= 2) { hash += (uint64_t)l2(p) * k3; p += 2; hash ^= rotr64(hash, 48) * k1; }
  if (len - p >= 1) { hash += (uint64_t)l1(p) * k3; hash ^= rotr64(hash, 37) * k1; }
  hash ^= rotr64(hash, 28);
  hash *= k0;
  hash ^= rotr64(hash, 29);
  return hash;
}

// metro64 over bytes at an arbitrary (unaligned) address.
VN_HD uint64_t metro64(const uint8_t* b, uint32_t len, uint64_t seed) {
  auto l1 = [b](uint32_t o) -> uint64_t { return b[o]; };
  auto l2 = [b](uint32_t o) -> uint64_t { return (uint64_t)b[o] | ((uint64_t)b[o + 1] << 8); };
  auto l4 = [b](uint32_t o) -> uint64_t {
    return (uint64_t)b[o] | ((uint64_t)b[o + 1] << 8) | ((uint64_t)b[o + 2] << 16) | ((uint64_t)b[o + 3] << 24);
  };
  auto l8 = [l4](uint32_t o) -> uint64_t { return l4(o) | (l4(o + 4) << 32); };
  return metro64_impl(len, seed, l8, l4, l2, l1);
}

// encodeHash(x, p=14, pp=25)
VN_HD uint32_t encode_hash(uint64_t x) {
  uint32_t idx = (uint32_t)(x >> (64 - kHllPP));                       // bextr(x, 39, 25)
  if (((x >> (64 - kHllPP)) & ((1ull << (kHllPP - kHllP)) - 1)) == 0) {  // bextr(x, 39, 11)
    uint64_t low = x & ((1ull << (64 - kHllPP)) - 1);                   // bextr(x, 0, 39)
    uint64_t zeros = clz64((low << kHllPP) | ((1ull << kHllPP) - 1)) + 1;
    return (idx << 7) | (uint32_t)(zeros << 1) | 1u;
  }
  return idx << 1;
}

// decodeHash(k, p=14, pp=25) -> (register index, rho)
VN_HD void decode_hash(uint32_t k, uint32_t* idx, uint32_t* r) {
  if (k & 1) {
    *r = ((k >> 1) & 63u) + (kHllPP - kHllP);
    *idx = (k >> (32 - kHllP)) & (kHllM - 1);
  } else {
    *r = (uint32_t)(clz64((uint64_t)(uint32_t)(k << (32 - kHllPP + kHllP - 1))) - 31);
    *idx = (k >> (kHllPP - kHllP + 1)) & (kHllM - 1);
  }
}

// varint byte length of a compressedList delta (compressed.go:167-173)
VN_HD uint32_t varint_len(uint32_t d) {
  uint32_t n = 1;
  while (d & 0xffffff80u) { d >>= 7; n++; }
  return n;
}

}  // namespace vn
