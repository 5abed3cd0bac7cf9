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

struct FeistelPerm {
  uint32_t key[4];
  uint32_t mask, n;
  int half;
  __device__ __forceinline__ void init(uint64_t seed, int epoch, uint32_t N) {
    n = N;
    int bits = 1;
    while ((1u << bits) < N) ++bits;
    bits += bits & 1;
    half = bits / 2;
    mask = (1u << half) - 1u;
    const uint64_t base = feistel_splitmix64(seed ^ feistel_splitmix64((uint64_t)epoch + 0x1234567ull));
#pragma unroll
    for (int r = 0; r < 4; ++r) key[r] = (uint32_t)feistel_splitmix64(base + r);
  }
  __device__ __forceinline__ uint32_t operator()(uint32_t x) const {
    do {
      uint32_t L = x >> half, R = x & mask;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t F = feistel_mix32(R ^ key[r]) & mask;
        const uint32_t nL = R;
        R = L ^ F;
        L = nL;
      }
      x = (L << half) | R;
    } while (x >= n);
    return x;
  }
};

// this rank's index list of `epoch`: out[i] = perm((rank + W*i) mod N), i < num_samples
__device__ __forceinline__ void rank_epoch_indices(int32_t* out, uint32_t N, int W, int rank, int num_samples,
                                                   uint64_t seed, int epoch, int shuffle, int tid, int nt) {
  FeistelPerm p;
  p.init(seed, epoch, N);
  for (int i = tid; i < num_samples; i += nt) {
    const uint32_t pos = (uint32_t)(((uint64_t)rank + (uint64_t)W * (uint64_t)i) % N);
    out[i] = (int32_t)(shuffle ? p(pos) : pos);
  }
}

// The epoch's list from a caller-provided index array (e.g. the host's torch-
// identical DistributedSampler order) when `given` is set, else the Feistel one.
__device__ __forceinline__ void rank_epoch_indices_or(const int32_t* given, int32_t* out, uint32_t N, int W, int rank,
                                                      int num_samples, uint64_t seed, int epoch, int shuffle, int tid,
                                                      int nt) {
  if (given != nullptr) {
    for (int i = tid; i < num_samples; i += nt) out[i] = given[i];
  } else {
    rank_epoch_indices(out, N, W, rank, num_samples, seed, epoch, shuffle, tid, nt);
  }
}

}  // namespace ptdt
