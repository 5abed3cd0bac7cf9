// Device-side DistributedSampler permutation (keyed Feistel bijection of
// [0, N) with cycle walking), shared by the standalone sampler kernel
// (rng.hip) and the persistent DDP step engine (fused_mlp.hip). Host model:
// pytorch_distributed_training_tutorials_amd/data/device_sampler.py.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptdt {

__device__ __forceinline__ uint32_t feistel_mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x7feb352dU; h ^= h >> 15; h *= 0x846ca68bU; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint64_t feistel_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Keyed 4-round Feistel bijection of [0, 2^bits), bits = ceil(log2 N), cycle-walked
// into [0, N). Unbalanced split (L: bits - hb, R: hb = bits / 2 bits; the rounds
// alternate L ^= F(R), R ^= F(L)) so the domain is the next power of two of N, not
// the next even power: at most half the draws walk again (none for N = 2^k), which
// bounds the divergence of a wave's cycle walks.
struct FeistelPerm {
  uint32_t key[4];
  uint32_t maskL, maskR, n;
  int hb;
  __device__ __forceinline__ void init(uint64_t seed, int epoch, uint32_t N) {
    n = N;
    int bits = 1;
    while ((1u << bits) < N) ++bits;
    hb = bits / 2;
    maskR = (1u << hb) - 1u;
    maskL = (1u << (bits - hb)) - 1u;
    const uint64_t base = feistel_splitmix64(seed ^ feistel_splitmix64((uint64_t)epoch + 0x1234567ull));
#pragma unroll
    for (int r = 0; r < 4; ++r) key[r] = (uint32_t)feistel_splitmix64(base + r);
  }
  __device__ __forceinline__ uint32_t operator()(uint32_t x) const {
    do {
      uint32_t L = x >> hb, R = x & maskR;
      L ^= feistel_mix32(R ^ key[0]) & maskL;
      R ^= feistel_mix32(L ^ key[1]) & maskR;
      L ^= feistel_mix32(R ^ key[2]) & maskL;
      R ^= feistel_mix32(L ^ key[3]) & maskR;
      x = (L << hb) | R;
    } while (x >= n);
    return x;
  }
};

// this rank's index list of `epoch`: out[i] = perm((rank + W*i) mod N), i < num_samples
__device__ __forceinline__ void rank_epoch_indices(int32_t* out, uint32_t N, int W, int rank, int num_samples,
                                                   uint64_t seed, int epoch, int shuffle, int tid, int nt) {
  FeistelPerm p;
  p.init(seed, epoch, N);
  // One 64-bit remainder per thread, then the wrap is a subtraction: a
  // remainder per entry (a software division loop) made this list ~14 us of
  // every persistent launch's prologue.
  uint32_t pos = (uint32_t)(((uint64_t)rank + (uint64_t)W * (uint64_t)tid) % N);  // once per thread
  const uint32_t step = (uint32_t)(((uint64_t)W * (uint64_t)nt) % N);
  for (int i = tid; i < num_samples; i += nt) {
    out[i] = (int32_t)(shuffle ? p(pos) : pos);
    pos += step;  // both < N: one conditional subtraction
    pos = pos >= N ? pos - N : pos;
  }
}

// Launch-to-launch cache of the epoch lists (global memory, owned by the
// caller's launch plan, fixed sampler parameters): slot e&1 holds epoch tag[e&1].
// A persistent launch copies a cached list instead of recomputing it, so the
// permutation is computed once per epoch however the steps are split into
// launches. The builder writes the tag only after every entry is written
// (the caller publishes it after its next barrier; readers are later launches).
struct ListCache {
  int32_t* lists;  // [2][stride], or nullptr: no cache
  int32_t* tag;    // [2] epoch held by each slot (-1: empty)
  int stride;
};

// The epoch's list from a caller-provided index array (e.g. the host's torch-
// identical DistributedSampler order) when `given` is set, else from the cache
// when it holds `epoch`, else the Feistel one (also written to the cache).
// Copy of a global list into LDS with every load in flight at once (up to
// kListSpec entries per thread): the plain loop waited for each unrolled group of
// 4 loads, two global round trips for 8 entries per thread, on the path to step 0.
constexpr int kListSpec = 16;
__device__ __forceinline__ void list_load(const int32_t* src, int num_samples, int tid, int nt, int32_t (&v)[kListSpec]) {
#pragma unroll
  for (int u = 0; u < kListSpec; ++u) {
    const int i = tid + u * nt;
    v[u] = i < num_samples ? src[i] : 0;
  }
}
__device__ __forceinline__ void list_store(int32_t* out, int num_samples, int tid, int nt, const int32_t (&v)[kListSpec]) {
#pragma unroll
  for (int u = 0; u < kListSpec; ++u) {
    const int i = tid + u * nt;
    if (i < num_samples) out[i] = v[u];
  }
}

__device__ __forceinline__ void rank_epoch_indices_or(const int32_t* given, int32_t* out, uint32_t N, int W, int rank,
                                                      int num_samples, uint64_t seed, int epoch, int shuffle, int tid,
                                                      int nt, const ListCache& lc = ListCache{nullptr, nullptr, 0}) {
  const bool spec = num_samples <= kListSpec * nt;
  if (given != nullptr) {
    if (spec) {
      int32_t v[kListSpec];
      list_load(given, num_samples, tid, nt, v);
      list_store(out, num_samples, tid, nt, v);
    } else {
      for (int i = tid; i < num_samples; i += nt) out[i] = given[i];
    }
    return;
  }
  if (lc.lists != nullptr) {
    // the slot's entries are read together with its tag (speculatively: the slot is
    // allocated whatever epoch it holds), one round trip on a hit
    const int32_t* src = lc.lists + (epoch & 1) * lc.stride;
    const int tag = lc.tag[epoch & 1];
    if (spec) {
      int32_t v[kListSpec];
      list_load(src, num_samples, tid, nt, v);
      if (__builtin_amdgcn_readfirstlane(tag) == epoch) {
        list_store(out, num_samples, tid, nt, v);
        return;
      }
    } else if (__builtin_amdgcn_readfirstlane(tag) == epoch) {
      for (int i = tid; i < num_samples; i += nt) out[i] = src[i];
      return;
    }
  }
  if (lc.lists != nullptr && tid == 0) lc.tag[epoch & 1] = -1;  // slot being overwritten until published
  rank_epoch_indices(out, N, W, rank, num_samples, seed, epoch, shuffle, tid, nt);
  if (lc.lists != nullptr) {
    int32_t* dst = lc.lists + (epoch & 1) * lc.stride;
    for (int i = tid; i < num_samples; i += nt) dst[i] = out[i];
  }
}
// Epochs e and e + 1 into out0 / out1: rank_epoch_indices_or twice, except that with the cache
// and no given lists both slots' entries and tags are loaded together (one round trip for two hits
// instead of two in a row on the path to step 0).
__device__ __forceinline__ void rank_epoch_indices_or2(const int32_t* given0, int32_t* out0, const int32_t* given1,
                                                       int32_t* out1, uint32_t N, int W, int rank, int num_samples,
                                                       uint64_t seed, int e, int shuffle, int tid, int nt,
                                                       const ListCache& lc) {
  if (given0 != nullptr || given1 != nullptr || lc.lists == nullptr || num_samples > kListSpec * nt) {
    rank_epoch_indices_or(given0, out0, N, W, rank, num_samples, seed, e, shuffle, tid, nt, lc);
    rank_epoch_indices_or(given1, out1, N, W, rank, num_samples, seed, e + 1, shuffle, tid, nt, lc);
    return;
  }
  const int32_t* const src0 = lc.lists + (e & 1) * lc.stride;
  const int32_t* const src1 = lc.lists + ((e + 1) & 1) * lc.stride;
  const int tag0 = lc.tag[e & 1], tag1 = lc.tag[(e + 1) & 1];
  int32_t v0[kListSpec], v1[kListSpec];
  list_load(src0, num_samples, tid, nt, v0);
  list_load(src1, num_samples, tid, nt, v1);
  const bool hit0 = __builtin_amdgcn_readfirstlane(tag0) == e, hit1 = __builtin_amdgcn_readfirstlane(tag1) == e + 1;
  if (hit0) list_store(out0, num_samples, tid, nt, v0);
  if (hit1) list_store(out1, num_samples, tid, nt, v1);
  if (!hit0) rank_epoch_indices_or(nullptr, out0, N, W, rank, num_samples, seed, e, shuffle, tid, nt, lc);
  if (!hit1) rank_epoch_indices_or(nullptr, out1, N, W, rank, num_samples, seed, e + 1, shuffle, tid, nt, lc);
}
// Publish `epoch` as cached (one thread, after every builder thread's writes).
__device__ __forceinline__ void list_cache_publish(const ListCache& lc, int epoch) {
  if (lc.lists != nullptr) lc.tag[epoch & 1] = epoch;
}

}  // namespace ptdt
