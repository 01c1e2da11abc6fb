/*
 * veneur_amd_synth.h -- deterministic synthetic DogStatsD-shaped streams (bench / tests).
 *
 * Not part of the reference boundary: this generates the already-parsed UDPMetric
 * batches (samplers/parser.go:21-43) that BASELINE.md's configs C1..C4 describe, so the
 * engine, the CPU oracle and the CPU baseline consume identical inputs.  Counter-based
 * RNG (splitmix64 of the sample index), so the output does not depend on thread count.
 */
#ifndef VENEUR_AMD_SYNTH_H
#define VENEUR_AMD_SYNTH_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t seed;
  uint32_t n_keys;            /* key universe "k%07u" */
  double zipf_s;              /* key popularity exponent (0 = uniform) */
  double mix[4];              /* class share by key: counter, gauge, histogram/timer, set */
  uint64_t n_samples;         /* samples generated for this shard */
  uint32_t shard, n_shards;   /* keep keys with FNV-1a digest % n_shards == shard */
  uint64_t member_universe;   /* set members "m%010llu" uniform in [0, universe) */
  double rate_half, rate_tenth; /* share of samples at rate 0.5 / 0.1 (others 1.0) */
  double histo_mu, histo_sigma; /* lognormal timer values (ms) */
  int threads;                /* 0 = hardware concurrency (capped at 16) */
} vn_synth_config;

typedef struct {
  uint32_t n_slots[4];
  uint64_t n[4];
  uint32_t* c_slot; double* c_val; float* c_rate;
  uint32_t* g_slot; double* g_val;
  uint32_t* h_slot; double* h_val; float* h_rate;
  uint32_t* s_slot; uint32_t* s_off; uint8_t* s_bytes; uint64_t s_nbytes;
  uint32_t* key_of_slot[4];   /* key id of every class-local slot */
  uint32_t* digest_of_slot[4];/* FNV-1a-32(name||type||"") of every slot */
} vn_synth_out;

int vn_synth_generate(const vn_synth_config* cfg, vn_synth_out* out);
void vn_synth_free(vn_synth_out* out);

#ifdef __cplusplus
}
#endif
#endif
