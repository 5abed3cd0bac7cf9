// Host-side launch API of every gfx950 kernel in this framework.
//
// The kernels are compiled by hipcc without any torch headers (fast, torch-ABI
// independent); csrc/bindings.cpp wraps them for at::Tensor. Every launcher
// takes an explicit hipStream_t and never allocates, copies host<->device or
// synchronises, so all of them can be captured into a hipGraph.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../comm/xgmi.h"

namespace ptdt {

// kF16 is accepted only where a launcher says so (the LLM.int8 pieces); elsewhere
// "not kF32" means bf16.
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

// --------------------------------------------------------------------------
// Fused small-MLP train step (csrc/kernels/fused_mlp.hip).
//
// One workgroup runs the whole per-rank step of a Linear[-ReLU-Linear] model
// for the DDP toy workloads (reference ddp_gpus.py:34-39, Linear(20,1)+CE):
// on-device batch gather by sampler indices -> forward -> loss -> backward ->
// gradients written (pre-scaled by 1/world_size) straight into the flat DDP
// bucket. Optionally it first applies the pending SGD update of the previous
// step from the (already all-reduced) bucket ("deferred update"), which folds
// the optimizer kernel into the next step's launch.
enum LossKind : int { kLossCESoft = 0, kLossCEIndex = 1, kLossMSE = 2 };

struct FusedMlpArgs {
  const float* X;        // [N, Din] device-resident dataset
  const float* Yf;       // [N, Dout] float targets (CE soft / MSE), or nullptr
  const int64_t* Yi;     // [N] class indices (CE index), or nullptr
  const int32_t* idx;    // [B] dataset rows of this step; nullptr => rows 0..B-1
  float* P;              // flat params [W1 H*Din | b1 H | W2 Dout*H | b2 Dout]; H==0: [W Dout*Din | b Dout]
  float* G;              // flat grads, same layout (the DDP bucket)
  float* mom;            // SGD momentum buffer (same layout) or nullptr
  int32_t* opt_step;     // device step counter for momentum init (may be nullptr)
  float* loss_out;       // [1] mean loss of this step
  int B, Din, H, Dout;
  int ldx;               // row stride of X in elements (0: Din)
  int x_padded;          // columns [Din, ldx) of X are zero (lets the wave engine read whole lane chunks)
  int loss_kind;
  int ignore_index;      // CE index: rows with this label are skipped (torch default -100)
  int has_bias;
  float grad_scale;      // 1/world_size (DDP pre-division)
  int accumulate;        // 1: G += grads (no_sync accumulation), 0: G = grads
  // SGD update folded into the step: update_mode 0 = none, 1 = "pre" (apply the
  // previous step's update from the already all-reduced bucket before the
  // forward), 2 = "post" (in-kernel xGMI all-reduce, then update this step).
  int update_mode;
  float lr, momentum, dampening, weight_decay;
  int nesterov;
  XgmiArgs ar;           // in-kernel one-shot all-reduce (ar.world == 0: off; needs update_mode 2 or 0)
};
hipError_t fused_mlp_step(const FusedMlpArgs& a, hipStream_t s);

// Persistent DDP step engine: ONE launch runs `n_steps` full DDP steps of the
// same model with parameters, momentum and the epoch's sampler indices kept
// resident in LDS; per step: gather batch (by the device sampler's index list,
// recomputed in-kernel at every epoch start) -> fwd/loss/bwd -> in-kernel
// all-reduce (xGMI one-shot; identity at world 1) -> SGD update. Uses
// FusedMlpArgs (update_mode must be 2; idx/loss_out unused) plus:
struct PersistArgs {
  int n_steps;
  int N;                 // dataset rows
  int W, rank;           // sampler sharding (== all-reduce world / rank)
  int num_samples;       // rows per rank per epoch (DistributedSampler num_samples)
  int shuffle;
  uint64_t seed;
  int32_t* cursor;       // device [epoch, step_in_epoch]; advanced by the kernel
  float* losses;         // [n_steps] per-step mean loss
  int stamps_n;          // elements of stamps (the TP engine adds per-wave barrier waits at [9 + w])
  int64_t* stamps;       // optional [9] diagnostic phase timers (s_memtime cycles, thread 0): prefetch issue,
                         // forward, loss, backward, all-reduce, sgd+land, epoch indices, total, realtime (100 MHz)
  int variant;           // kPersistAuto / kPersistWorkgroup / kPersistWave...
  int loss_ring;         // set by the launcher: the wave engine reduces losses in helper waves
  const int32_t* idx;    // optional [idx_epochs][num_samples] index lists of epochs idx_e0.. (e.g. torch's
                         // DistributedSampler orders; replace the in-kernel Feistel permutation). A launch
                         // must stay inside those epochs; list reads past them (stale prefetches) clamp.
  int idx_e0, idx_epochs;
  int64_t cursor_host_pos;  // the caller's view of the cursor (epoch * steps_per_epoch + step), or -1
  int32_t* lcache;       // optional [2][al4(num_samples)] launch-to-launch epoch-list cache (sampler.h ListCache)
  int32_t* ltag;         // its [2] epoch tags (-1: empty); both null: every launch recomputes its lists
  // host-asserted start position (PersistentPlan.launch_at): when has_start is set the
  // caller guarantees the device cursor holds (start_e, start_j), and the wave/TP engines
  // take it from the kernel arguments instead of a dependent load at kernel entry
  int has_start, start_e, start_j;
  // optional launch timeline (tools/driver_timeline.py): thread 0 stores the 100 MHz realtime
  // counter at [0] kernel entry, [1] past the prologue barrier, [2] after the last step,
  // [3] after the final parameter / cursor stores. May point at host-mapped memory.
  int64_t* tl;
};
// Engine choice: the register-resident single-wave engine (linear_wave.hip) runs
// Linear(Din, Dout) models with B <= 64 and small Dout; everything else runs the
// LDS workgroup engine (fused_mlp.hip). kPersistAuto picks the wave engine when
// it supports the configuration.
// kPersistWaveRows / kPersistWaveF restrict the wave engine to one lane-layout
// family (row groups across DPP rows / feature groups across DPP rows).
#ifndef PTDT_WAVE_PREFETCH
#define PTDT_WAVE_PREFETCH 3
#endif
constexpr int kWavePrefetch = PTDT_WAVE_PREFETCH;  // batches in flight in the wave engine (register buffers)
// FusedMlpArgs::ldx of an engine-choice query (persistent_engine()): any row stride, the caller pads
// X rows to the chosen layout's width
constexpr int kWaveLdxAny = 1 << 20;
// LDS stride of one epoch index list in the wave engines: S batches of B entries plus up to 64
// padding entries (layout F reads row slots rho * 16 + i < 16 R <= 64 of the last batch unclamped)
__host__ __device__ __forceinline__ int wave_list_stride(int num_samples, int B) {
  return (((num_samples + B - 1) / B) * B + 64 + 3) & ~3;
}
// kPersistMfma: the workgroup engine with the 4-wave MFMA step body for
// Linear-ReLU-Linear (B <= 32, Din <= 32, H in 16..64 step 16, Dout <= 16);
// kPersistAuto picks it for those shapes.
// kPersistTp: Linear-ReLU-Linear tensor-parallel across the waves of one
// workgroup (mlp_tp.hip: each wave owns 16 hidden units, every product on
// MFMA, one barrier per step); kPersistAuto picks it for B <= 32, Din <= 32,
// H in 16..64 step 16, Dout <= 16.
// kPersistTpBf16: the same engine on bf16 operands (torch.autocast(bfloat16) rounding points,
// fp32 master weights and SGD; v_mfma_f32_16x16x32_bf16 / 16x16x16_bf16). Never picked by
// kPersistAuto: bf16 is requested explicitly (FusedMLPStep(dtype="bf16"), bench --dtype bf16).
enum PersistVariant : int {
  kPersistAuto = 0, kPersistWorkgroup = 1, kPersistWave = 2, kPersistWaveRows = 3, kPersistWaveF = 4,
  kPersistMfma = 5, kPersistTp = 6, kPersistTpBf16 = 7
};
// The caller-provided list of `epoch` (clamped into the provided range), or nullptr.
__device__ __forceinline__ const int32_t* given_list(const PersistArgs& p, int epoch) {
  if (p.idx == nullptr) return nullptr;
  int k = epoch - p.idx_e0;
  k = k < 0 ? 0 : (k >= p.idx_epochs ? p.idx_epochs - 1 : k);
  return p.idx + (int64_t)k * p.num_samples;
}
hipError_t fused_mlp_persistent(const FusedMlpArgs& a, const PersistArgs& p, hipStream_t s);
// A persistent launch resolved once (engine choice, kernel, LDS size, argument
// checks): relaunching it only sets n_steps (and the explicit-list cursor) and
// calls hipLaunchKernel, so a short run pays no per-call planning.
struct PersistLaunch {
  const void* fn = nullptr;
  int threads = 0;
  size_t lds = 0;
  FusedMlpArgs a{};
  PersistArgs p{};
  int64_t host_ns[2] = {0, 0};  // CLOCK_MONOTONIC right before / after the last hipLaunchKernel
};
// Timeline probe support (timeline.hip): thread 0 of wave 0 writes the realtime counter.
__device__ __forceinline__ void tl_mark(int64_t* tl, int k) {
  if (tl != nullptr && threadIdx.x == 0)
    __hip_atomic_store(tl + k, (int64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Host <-> device clock calibration: a 1-thread kernel answers n host pings (flag[k] = k + 1)
// with its realtime counter in out[k]; host-mapped buffers. Returns per ping
// (host ns before the flag store, host ns when the answer was seen, device ticks).
hipError_t clock_calibrate(int n, int64_t* host_set, int64_t* host_seen, int64_t* dev_ticks);
hipError_t fused_mlp_persistent_prepare(const FusedMlpArgs& a, const PersistArgs& p, PersistLaunch* out);
hipError_t persistent_launch(PersistLaunch& L, int n_steps, int64_t cursor_host_pos, hipStream_t s,
                             int start_e = -1, int start_j = 0);
bool linear_wave_supported(const FusedMlpArgs& a, const PersistArgs& p);
bool mlp_mfma_persistent_supported(const FusedMlpArgs& a, const PersistArgs& p);
bool mlp_tp_supported(const FusedMlpArgs& a, const PersistArgs& p);
hipError_t mlp_tp_prepare(const FusedMlpArgs& a, const PersistArgs& p, PersistLaunch* out);
// lane layout the wave engine picks: L lanes per row, R rows per lane group, kp features per lane
void linear_wave_layout(const FusedMlpArgs& a, const PersistArgs& p, int* L, int* R, int* kp);
hipError_t linear_wave_persistent(const FusedMlpArgs& a, const PersistArgs& p, hipStream_t s);
hipError_t linear_wave_prepare(const FusedMlpArgs& a, const PersistArgs& p, PersistLaunch* out);
size_t fused_mlp_persistent_lds_bytes(int B, int Din, int H, int Dout, int num_samples, int world);
// LDS bytes the step needs (host check against the 160 KiB per-CU budget).
size_t fused_mlp_lds_bytes(int B, int Din, int H, int Dout);

// torch-identical DistributedSampler epoch orders on the GPU (torch_perm.hip):
// out[e][i] = torch.randperm(n, generator=manual_seed(seeds[e]))[(rank + W*i) % n]
// for i < num_samples, one workgroup per epoch. ws: int32[n_epochs][4n] global
// scratch, needed only when 4n ints exceed the LDS budget (torch_perm_lds_bytes).
hipError_t torch_perm(const int64_t* seeds, int n_epochs, int n, int W, int rank, int num_samples, int32_t* out,
                      int out_stride, int32_t* ws, hipStream_t s);
size_t torch_perm_lds_bytes(int n);

// --------------------------------------------------------------------------
// Optimizers on flat buffers and multi-tensor lists (csrc/kernels/optim.hip).
// torch.optim.SGD semantics: d = g + wd*p; buf = (first ? d : mu*buf + (1-damp)*d);
// d = nesterov ? d + mu*buf : buf; p -= lr*d.
hipError_t sgd_flat(float* p, const float* g, float* mom, int32_t* step, int64_t n, float lr,
                    float momentum, float dampening, float weight_decay, int nesterov,
                    float grad_scale, hipStream_t s);
// Adam/AdamW; step is a device counter already incremented for this step.
hipError_t adam_flat(float* p, const float* g, float* m, float* v, const int32_t* step, int64_t n,
                     float lr, float beta1, float beta2, float eps, float weight_decay,
                     int decoupled, float grad_scale, hipStream_t s);

constexpr int kMaxTensorsPerLaunch = 32;
struct TensorList {
  int n;                                   // tensors in this launch
  int64_t numel[kMaxTensorsPerLaunch];
  void* p[kMaxTensorsPerLaunch];           // param (f32 or bf16, see dtype)
  const void* g[kMaxTensorsPerLaunch];     // grad (same dtype as param)
  float* s1[kMaxTensorsPerLaunch];         // momentum / exp_avg (f32) or nullptr
  float* s2[kMaxTensorsPerLaunch];         // exp_avg_sq (f32) or nullptr; SGD on f32 params: optional bf16
                                           // shadow of the updated param (uint16_t*), the autocast weight copy
};
hipError_t sgd_multi(const TensorList& tl, int dtype, int32_t* step, float lr, float momentum,
                     float dampening, float weight_decay, int nesterov, float grad_scale,
                     hipStream_t s);
hipError_t adam_multi(const TensorList& tl, int dtype, const int32_t* step, float lr, float beta1,
                      float beta2, float eps, float weight_decay, int decoupled, float grad_scale,
                      hipStream_t s);
// dst[i] = src_i * scale over a list (bucket pack) or the reverse (unpack).
struct CopyList {
  int n;
  int64_t numel[kMaxTensorsPerLaunch];
  int64_t offset[kMaxTensorsPerLaunch];    // element offset inside the flat buffer
  void* t[kMaxTensorsPerLaunch];           // the per-parameter tensors
};
hipError_t bucket_pack(const CopyList& cl, void* flat, int dtype, float scale, hipStream_t s);
hipError_t bucket_unpack(const CopyList& cl, const void* flat, int dtype, float scale, hipStream_t s);
hipError_t scale_inplace(void* x, int64_t n, int dtype, float scale, hipStream_t s);
// tl.p[t] (f32) = tl.g[t] (bf16) elementwise, every tensor dense with matching layouts
hipError_t cast_bf16_f32_multi(const TensorList& tl, hipStream_t s);

// --------------------------------------------------------------------------
// Losses (csrc/kernels/loss.hip). Row-wise log-softmax CE (soft or index
// targets, mean reduction) and MSE mean. Forward writes the mean loss and the
// per-row logsumexp; backward writes dlogits = g_out * dL/dlogits.
hipError_t ce_forward(const void* logits, int dtype, const float* soft, const int64_t* index,
                      int B, int C, int ignore_index, float label_smoothing, float* loss,
                      float* lse, float* valid_count, hipStream_t s);
hipError_t ce_backward(const void* logits, int dtype, const float* soft, const int64_t* index,
                       const float* lse, const float* valid_count, const float* grad_out, int B,
                       int C, int ignore_index, float label_smoothing, void* dlogits,
                       hipStream_t s);
hipError_t mse_forward(const void* x, const void* y, int dtype, int64_t n, float* loss,
                       hipStream_t s);
hipError_t mse_backward(const void* x, const void* y, int dtype, int64_t n, const float* grad_out,
                        void* dx, void* dy, hipStream_t s);

// --------------------------------------------------------------------------
// GEMM on MFMA (csrc/kernels/gemm.hip).
// C[M,N] = alpha * A[M,K] * B[K,N] (+ beta*C) (+ bias[N]) (ReLU), A and B addressed
// by (row, col) strides so NN/NT/TN layouts need no transposed copies.
// f32 operands use v_mfma_f32_32x32x2_f32 (exact fp32), bf16 operands
// v_mfma_f32_16x16x32_bf16; accumulation is always fp32.
struct GemmArgs {
  int M, N, K;
  const void* A; int64_t sam, sak;      // A(m,k) = A[m*sam + k*sak]
  const void* B; int64_t sbk, sbn;      // B(k,n) = B[k*sbk + n*sbn]
  void* C; int64_t scm, scn;            // C(m,n)
  int in_dtype, out_dtype;
  const void* bias;                     // [N] (in out_dtype precision rules: f32 or bf16), or nullptr
  int bias_dtype;
  const void* amask; int64_t smm, smk;  // optional ReLU mask on A: A(m,k) used only where mask(m,k) > 0
  int relu;                             // ReLU epilogue
  float alpha, beta;                    // beta!=0 reads C (accumulate)
  float* colsum_out;                    // optional: colsum_out[m] += sum_k A(m,k) (masked) -> bias grads
  int split_k;                          // >1: fp32 atomics into C (C must be f32 and pre-zeroed by caller)
};
hipError_t gemm(const GemmArgs& g, hipStream_t s);

// Throughput bf16 GEMM (csrc/kernels/gemm_big.hip): C = alpha*A.Bt^T (+beta*C)(+bias)(ReLU),
// A [M,K] and Bt [N,K] both K-contiguous bf16, C f32 or bf16 with row stride ldc.
struct BigGemmArgs {
  int M, N, K;
  const void* A; int64_t lda;
  const void* Bt; int64_t ldb;
  void* C; int64_t ldc;
  int out_dtype;
  const void* bias; int bias_dtype;
  int relu;
  float alpha, beta;
  int sched;    // 0: read-then-multiply per K-tile, 1: ping-pong wave pairs, 2: ping-pong fed from a 10-piece LDS ring, 3: 8-phase quadrant schedule, 4: 3 with grouped tile order (default, 256 tile), 5 / 6: group of 4 / 16 rows
  int tile;     // 256: 256x256 block tile (8 waves), 128: 128x128 (4 waves, 2 workgroups per CU)
  int split_k;  // >1: K split over gridDim.y, fp32 atomics into a pre-zeroed f32 C (no ReLU/beta)
};
bool gemm_bf16_big_supported(int M, int N, int K, int64_t lda, int64_t ldb, const void* A, const void* Bt);
hipError_t gemm_bf16_big(const BigGemmArgs& g, hipStream_t s);

// Elementwise helpers (csrc/kernels/elementwise.hip)
hipError_t relu_backward(const void* dy, const void* y, void* dx, int dtype, int64_t n, hipStream_t s);
// NHWC [npix, 3] (f32 / bf16) -> NHWC [npix, 4] bf16, 4th channel zero (RGB stem padding)
hipError_t rgb4_pack(const void* x, int dtype, uint16_t* y, int64_t npix, hipStream_t s);
// out[0] = sum of all n elements (fp32 accumulate, deterministic), one workgroup.
hipError_t sum_all(const void* x, int dtype, int64_t n, float* out, hipStream_t s);

// One-thread completion mark for a graph-captured collective (csrc/comm/rccl_comm.cpp):
// ++*ctr (device memory), then the new value is stored to the host-mapped mirror.
hipError_t comm_done_mark(uint64_t* ctr, uint64_t* host_mirror, hipStream_t s);
// Fixed-order column sums (deterministic; no atomics or memsets). nsplit > 1 needs a
// float workspace of nsplit * cols; col_sum_splits picks nsplit for a shape.
int col_sum_splits(int64_t rows, int64_t cols);
hipError_t col_sum(const void* x, int dtype, int64_t rows, int64_t cols, float* out, int accumulate, float* ws,
                   int nsplit, hipStream_t s);
hipError_t fill_f32(float* x, float v, int64_t n, hipStream_t s);
hipError_t cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s);
hipError_t cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t s);

// --------------------------------------------------------------------------
// Synthetic data on device (csrc/kernels/rng.hip): counter-based Philox4x32-10.
// dist 0 = uniform [0,1) (torch.rand-like), 1 = standard normal (Box-Muller).
hipError_t philox_fill(float* out, int64_t n, uint64_t seed, uint64_t offset, int dist,
                       hipStream_t s);
// one_hot[b, idx[b]] = 1, zeros elsewhere (reference NB03:958 scatter_).
hipError_t one_hot(const int64_t* idx, float* out, int B, int C, hipStream_t s);
// out[i, :] = src[idx[i], :] (device batch gather of a resident dataset).
hipError_t gather_rows(const void* src, const int32_t* idx, void* out, int64_t rows, int64_t cols,
                       int elem_bytes, hipStream_t s);

// Device-side DistributedSampler: out[i] = perm_e(rank + W*i mod N) for
// i < num_samples, where perm_e is a keyed Feistel bijection of [0, N)
// (cycle-walking) for epoch e. The epoch lives in device memory: the kernel
// computes epoch = *epoch_ptr + 1 and stores it back, so a hipGraph holding
// this kernel advances epochs by itself on every replay. Same sharding /
// padding semantics as torch's DistributedSampler (different permutation).
hipError_t device_sampler(int32_t* out, int64_t N, int W, int rank, int64_t num_samples, uint64_t seed,
                          int32_t* epoch_ptr, int shuffle, hipStream_t s);

// --------------------------------------------------------------------------
// Int8 weight-only quantization + GEMM (csrc/kernels/int8.hip), LLM.int8-style
// row-wise absmax (reference NB03:52-56 BitsAndBytesConfig(load_in_8bit)).
hipError_t quantize_rowwise_int8(const void* w, int dtype, int64_t rows, int64_t cols, int8_t* q,
                                 float* scale, hipStream_t s);
// y[M,N] = x[M,K] (bf16/f32) * dequant(q[N,K])^T (+bias), i8 weights dequantised in LDS
// into bf16 and multiplied on v_mfma_f32_16x16x32_bf16.
hipError_t int8_weight_gemm(const void* x, int x_dtype, const int8_t* q, const float* scale,
                            const void* bias, int M, int N, int K, void* y, int y_dtype,
                            hipStream_t s);

// LLM.int8 (csrc/kernels/int8_mm.hip): outlier columns (|x| > threshold), row-wise
// activation quantisation with them zeroed, int8 x int8 -> int32 MFMA GEMM with the
// dequantisation, the caller's outlier product (addend, f32 [M,N]) and bias in the epilogue.
// ws: K unsigned of scratch (the column maxima)
hipError_t int8_col_outliers(const void* x, int dtype, int M, int K, float threshold, uint8_t* mask, unsigned* ws,
                             hipStream_t s);
hipError_t int8_quant_rows(const void* x, int dtype, int M, int K, const uint8_t* mask, int8_t* q, float* scale,
                           hipStream_t s);
// x / y / bias dtypes: kF32, kBF16 or kF16. K % 128 == 0 and 16-B aligned operands take the
// LDS-staged 128x128-tile kernel (int8_mm_tiled_supported), other K % 16 == 0 the direct one.
hipError_t int8_mm(const int8_t* A, const float* sa, const int8_t* B, const float* sb, const float* addend,
                   const void* bias, int bias_dtype, int M, int N, int K, void* y, int y_dtype, hipStream_t s);
bool int8_mm_tiled_supported(int M, int N, int K);
// hipGraph editing before instantiation (graph_memset.hip): node-type census (counts[type] for
// type < ncounts; returns the node count, -1 on error) and memset nodes -> fill-kernel nodes
// (returns how many were replaced, -1 on error)
int graph_node_census(void* graph, int* counts, int ncounts);
int graph_replace_memsets(void* graph);
}  // namespace ptdt
#include <vector>
namespace ptdt {
int graph_memset_params(void* graph, std::vector<std::vector<int64_t>>* out);
hipError_t graph_memset_run(void* dst, uint32_t value, int esize, size_t width, size_t height, size_t pitch,
                            int reps, hipStream_t s);

// LLM.int8 decode path (csrc/kernels/int8_decode.hip): M <= 32 rows, K % 64 == 0, K <= kInt8DecodeMaxK.
// Outlier detection, activation quantisation and the int8 GEMV with the outlier columns fused, in two
// launches and no host read. ws: int8_decode_ws_bytes(M, K) bytes, 16-B aligned.
constexpr int kInt8DecodeMaxK = 16384;
size_t int8_decode_ws_bytes(int M, int K);
bool int8_decode_supported(int M, int N, int K);
// Wp: optional pre-shuffled copy of W (int8_decode_pack, int8_decode_packed_bytes(N, K) bytes) for
// contiguous weight loads in the GEMV; nullptr reads the row-major W.
hipError_t int8_decode(const void* x, int x_dtype, int M, int K, float threshold, const int8_t* W, const int8_t* Wp,
                       const float* sw, const void* bias, int bias_dtype, int N, void* y, int y_dtype, void* ws,
                       hipStream_t s);
size_t int8_decode_packed_bytes(int N, int K);
hipError_t int8_decode_pack(const int8_t* W, int N, int K, int8_t* Wp, hipStream_t s);

// BatchNorm(train stats applied) + ReLU fused epilogue over NCHW (csrc/kernels/elementwise.hip)
hipError_t bn_relu_apply(const void* x, int dtype, const float* scale, const float* shift, int64_t N,
                         int64_t C, int64_t HW, int relu, void* y, hipStream_t s);

// Training BatchNorm over channels-last [M, C] activations with ReLU / residual
// epilogues fused (csrc/kernels/batchnorm.hip). Statistics / coefficients are f32
// [C] device arrays; `tickets` is a zeroed int array (>= bn_num_tickets), re-armed
// by the kernels; `workspace` holds bn_workspace_floats floats.
struct BnParams {
  const float* weight; const float* bias;   // may be null (affine=False)
  float* running_mean; float* running_var;  // may be null (track_running_stats=False)
  int64_t* num_batches_tracked;             // may be null
  float momentum, eps;
  float* mean; float* invstd;               // saved for backward
  float* scale; float* shift;               // y = x*scale + shift
  int fence_handoff = 0;                    // A/B only (PTDT_BN_FENCE=1): the old release/acquire hand-off
};
struct BnFwdArgs {
  const void* x; const void* residual; void* y;  // residual may be null
  int dtype; int64_t M; int C; int relu;
  float* workspace; int* tickets;
  BnParams p;
  uint8_t* mask_out;  // relu + residual: the ReLU mask, one byte per 16-B vector (bit v: y > 0), or null
  int stats_ready;    // p.scale/shift already hold this batch's coefficients (gemm_bn_stats): apply pass only
};
// 1x1 convolution + BatchNorm batch statistics (gemm_big.hip gemm_bn_stats): C = A . Bt^T in bf16
// (bias/ReLU/beta unused) and the statistics of C's columns into p.mean/invstd/scale/shift, running
// stats updated. ws: gemm_bn_ws_floats(); tickets: gemm_bn_num_tickets() zeroed ints (re-armed).
struct GemmBnEpi {
  float* ws;
  int* tickets;
  int group;  // row tiles per merge group (host: gemm_bn_stats fills it)
  BnParams p;
};
int64_t gemm_bn_ws_floats(int M, int N, int tile);
int gemm_bn_num_tickets(int M, int N, int tile);
hipError_t gemm_bn_stats(const BigGemmArgs& g, GemmBnEpi e, hipStream_t s);
// Streaming variant for the memory-bound shapes (conv1x1_bn.hip): X [M, K] and W [N, K] bf16 with
// unit row strides K, Y [M, N] bf16; supported (K, N) pairs only; ws / tickets sized by the helpers.
bool conv1x1_bn_stream_supported(int K, int N);
int64_t conv1x1_bn_stream_ws_floats(int M, int K, int N);
int conv1x1_bn_stream_num_tickets(int M, int K, int N);
hipError_t conv1x1_bn_stream(const void* X, const void* W, void* Y, int M, int K, int N, GemmBnEpi e,
                             hipStream_t s);

struct BnBwdParams {
  const float* weight; const float* mean; const float* invstd;
  const float* scale; const float* shift;   // forward scale/shift: ReLU mask from x when y is null
  float* dweight; float* dbias;             // may be null
  float* coef_a; float* coef_b; float* coef_c;  // scratch [C] each
  int fence_handoff = 0;                    // A/B only (PTDT_BN_FENCE=1), as BnParams
};
struct BnBwdArgs {
  const void* dy; const void* x; const void* y;  // y: forward output (ReLU mask) or null: mask from x
  const void* dy2;                               // optional second gradient addend (dy + dy2), or null
  void* dx; void* dres;                          // dres (may be null): gradient of the residual = masked dy
  int dtype; int64_t M; int C; int relu;
  float* workspace; int* tickets;
  BnBwdParams p;
  const uint8_t* mask;  // the forward's mask_out (instead of y; needs dres), or null
  int reduce_only = 0;  // 1: the reduce pass only, writing the masked gradient g to dres (no dx): the
                        // consumer applies dx = A g + B x + C itself (conv1x1_bwd, coef_a/b/c)
};
int64_t bn_workspace_floats(int64_t M, int C, int dtype);
int bn_num_tickets(int C, int dtype);
hipError_t bn_forward_train(const BnFwdArgs& a, hipStream_t s);
hipError_t bn_backward(const BnBwdArgs& a, hipStream_t s);
// Backward of BN(conv1x1(x)) for the streaming shapes (csrc/kernels/conv1x1_bwd.hip): dY = A g + B y + C
// (coef = [A; B; C], 3 x N floats, from a reduce_only bn_backward) feeds dX = dY W and dW = dY^T X
// without storing dY. g, y: [M, N] bf16; x: [M, K]; w: [N, K]; dx: [M, K]; dw: [N, K] bf16.
bool conv1x1_bwd_supported(int K, int N);
int64_t conv1x1_bwd_ws_floats(int M, int K, int N);
hipError_t conv1x1_bwd(const void* g, const void* y, const void* x, const void* w, const float* coef, void* dx,
                       void* dw, float* ws, int M, int K, int N, hipStream_t s);
// y = ReLU?(x*scale + shift (+ residual)) per channel (eval-mode BN, or any affine epilogue)
hipError_t bn_apply(const void* x, const void* residual, void* y, int dtype, const float* scale, const float* shift,
                    int64_t M, int C, int relu, hipStream_t s);

// Max pooling over NHWC activations (csrc/kernels/pool.hip): argmax is one byte per
// output element (window offset dy*kw + dx), the backward a deterministic gather.
struct PoolArgs {
  int N, H, W, C, Ho, Wo;
  int kh, kw, sh, sw, ph, pw;
  // forward only, optional: every loaded x becomes ReLU?(x * scale[c] + shift[c]) rounded to x's type
  // before the max -- a training BatchNorm's apply pass folded into the pool that consumes it
  const float* scale = nullptr;
  const float* shift = nullptr;
  int relu = 0;
};
hipError_t maxpool2d_nhwc_forward(const void* x, void* y, uint8_t* argmax, int dtype, const PoolArgs& a,
                                  hipStream_t s);
hipError_t maxpool2d_nhwc_backward(const void* gy, const uint8_t* argmax, void* gx, int dtype, const PoolArgs& a,
                                   hipStream_t s);

}  // namespace ptdt
