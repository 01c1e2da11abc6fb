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

#include "veneur_amd.h"

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

/* The C4 stream, generated in HBM by the GPU: one global stream of n_samples records over
 * n_keys keys (Zipf popularity, alias-method draws; the classes and digests of the keys as
 * vn_synth_generate), of which this rank keeps its own -- keys routed by digest % nranks
 * (server.go:655), split keys dealt round-robin by their window arrival index (record j of a
 * split key to rank j % nranks).  Local slots per class: the rank's own keys in ascending key
 * id, then the class's split keys in list order (split key i at split_slot0[class] + i).  Split
 * counters come out in `batch` at their local slot; split histograms and sets in `split`. */
typedef struct {
  uint64_t seed;
  uint32_t n_keys;
  double zipf_s;
  double mix[4];
  uint64_t n_samples;           /* positions of the global stream */
  uint32_t rank, nranks;
  uint64_t member_universe;
  double rate_half, rate_tenth, histo_mu, histo_sigma;
  int device;
  uint32_t n_split[4];          /* split keys per class (gauges: 0) */
  const uint32_t* split_key[4]; /* their key ids (host arrays) */
} vn_synth_dev_config;

typedef struct {
  uint32_t n_slots[4];
  uint32_t split_slot0[4];
  uint32_t* key_of_slot[4];     /* host arrays */
  uint32_t* digest_of_slot[4];
  vn_batch batch;               /* device arrays (vn_ingest) */
  vn_split_batch split;         /* device arrays (vn_ingest_split) */
  uint64_t n_member_bytes, n_split_member_bytes;
  int64_t counter_sum;          /* this rank's sum of int64(value) * int64(float32(1 / rate)) */
  double histo_weight;          /* this rank's sum of histogram weights */
} vn_synth_dev_out;

int vn_synth_device(const vn_synth_dev_config* cfg, vn_synth_dev_out* out);
void vn_synth_device_free(vn_synth_dev_out* out);
/* record count of every key over the first n_positions of the stream (hot-key detection) */
int vn_synth_key_counts(const vn_synth_dev_config* cfg, uint64_t n_positions, uint32_t* counts /* n_keys */);

/* C5 (BASELINE configs[4]): the local flush windows of hosts [host0, host0 + n_hosts) of a
 * global aggregator's fleet, generated in HBM.  Host h's histogram key k (< n_histo_keys) gets
 * 50 + (x % 101) timer samples (lognormal, mu 3.9 + 0.05 (h % 8), sigma 1; 10% at rate 0.5), its
 * set key k (< n_set_keys) min(20000, int(50 * Lomax(1.2)) + 1) member hashes (x a counter-based
 * draw of (seed, h, k)).  Records of host h, key k sit at local slot (h - host0) * n_keys + k,
 * host-major then key-major, each key's samples in draw order: ingested into one local engine of
 * n_hosts * n_keys slots per class and exported, they are every host's forwarded payloads. */
typedef struct {
  uint64_t seed;
  uint32_t host0, n_hosts, n_histo_keys, n_set_keys;
  int device;
} vn_synth_hosts_config;

typedef struct {
  uint64_t n_histo, n_set;
  uint32_t* h_slot;             /* device arrays, freed by vn_synth_hosts_free */
  double* h_val;
  float* h_rate;
  uint32_t* s_slot;
  uint64_t* s_hash;
} vn_synth_hosts_out;

int vn_synth_hosts_device(const vn_synth_hosts_config* cfg, vn_synth_hosts_out* out);
void vn_synth_hosts_free(vn_synth_hosts_out* out);

#ifdef __cplusplus
}
#endif
#endif
