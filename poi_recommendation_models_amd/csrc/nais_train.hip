// nais_train.hip -- gfx950 kernels + C-ABI for the NAIS_basic training step.
//
// Reference: get_NAIS_batch (batches.py:24-50) builds b = (1 + num_ng) * n rows that all share the
// user's n positives as their history; train_NAIS (run.py:91-109) then runs model.forward in train
// mode (Dropout(0.5) on W1 x + b1, model.py:22,71), BCELoss (model.py:21,96-97), backward and
// Adagrad (run.py:89,102-109).
//
// Per pair (row c, history item j), with x = h_j (.) t_c, u = W1 x + b1, v = u * m_cj (dropout
// factors m in {0, 1/(1-p)}), z = ReLU(v), a = w2 . z, e = exp(a) [h_j != t_c], s = h_j . t_c:
//   S_c = sum_j e, N_c = sum_j e s, logit_c = N_c / S_c^beta, pred_c = sigmoid(logit_c).
// Given g_c = dL/dlogit_c (from dL/dpred via the sigmoid), the backward of model.py:57-89 is
//   ds = g e / S^beta                      (dlogit/ds_cj)
//   da = ds (s - beta N / S)               (dlogit/de_cj times de/da = e)
//   du = da w2 [v > 0] * scale             (ReLU + dropout backward, scale = 1/(1-p) if kept)
//   dW1 += du x^T, db1 += du, dw2 += da z, dx = W1^T du, r = dx + ds
//   dh_j += r (.) t_c, dt_c += r (.) h_j.
// Both kernels recompute u from the embeddings (one exact-fp32 MFMA chain, as the scorer), so no
// [b, n, H] tensor is ever stored; dropout factors come from a counter hash of (seed, c*n+j, i),
// so the forward and backward launches see the same mask without storing it.
//
// MFMA layout (v_mfma_f32_32x32x2_f32, 32 rows per wave as the B/C columns):
//   forward  acc[hb] (32 hidden x 32 rows) += W1[hb block][K pair] x x[K pair][rows]
//   dx       dx[db]  (32 dims x 32 rows)   += W1^T[db block][K pair] x du[K pair][rows]
//            -- du is fed straight from the forward accumulator registers: K-step (hb, r) takes
//               hidden unit crow(hb, r, hh), so no data movement is needed. The forward K order
//               over embedding dims is chosen as the C layout of dx (kdim below), so the lane that
//               supplies x[dim] holds dx[dim] afterwards.
//   dW1      per item, the 128 rows of du and x go through LDS ([row][hidden], [row][dim]) and
//            each wave accumulates its 32x32 tiles of dW1 with K = the workgroup's 128 rows.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>
#include <stdint.h>

#include <algorithm>
#include <string>

#include "nais.h"
#include "nais_internal.h"
#include "nais_gx.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int TW = 4;               // waves per training workgroup (one per SIMD)
constexpr int TTHREADS = TW * 64;
constexpr int TROWS = TW * 32;      // batch rows per workgroup: 32 per wave (the MFMA columns)
constexpr int MAX_JS = 32;          // history items per slice (grid.y)

// Per-phase cycle accounting hooks of the backward kernels: no-ops in the product library. The
// timing build (scripts/probes/train_timing.hip) defines them -- s_memtime deltas per phase, summed
// into a device array that its nais_debug_train_cycles() reads (scripts/train_phases.py) -- and
// includes this file; the hooks never change a result.
#ifndef TSTART
#define TSTART() (void)0
#define TMARK(k) (void)0
#define TFLUSH() (void)0
#endif

__device__ __forceinline__ floatx16 mfma(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// row held in accumulator register r of 32-row block blk by lane half hh (32x32 C layout)
__device__ __forceinline__ int crow(int blk, int r, int hh) {
  return blk * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
}
// embedding dim carried by K-step s of the forward MFMA in lane half hh (= C layout of dx)
__device__ __forceinline__ int kdim(int s, int hh) { return crow(s >> 4, s & 15, hh); }
// first of the 4 consecutive dims of K-steps 4g..4g+3
__device__ __forceinline__ int kdim4(int g, int hh) { return 32 * (g >> 2) + 8 * (g & 3) + 4 * hh; }

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Dropout as in nn.Dropout(p) (model.py:22): keep with probability 1-p and scale by 1/(1-p).
// The draw for hidden unit i of pair (c, j) is a hash of (seed, c*n+j, i) -- same bits in every
// kernel, no mask storage. Distributionally the reference's Bernoulli mask, not its RNG stream
// (the parity tests inject the mask through nais_dropout_mask).
struct Drop {
  uint32_t s0, s1, thr;
  float scale;
  int on;
  __device__ __forceinline__ uint32_t key(uint32_t pair) const { return mix32(pair ^ s0); }
  __device__ __forceinline__ float factor(uint32_t k, int i) const {
    return mix32((k + uint32_t(i) * 0x9e3779b9u) ^ s1) >= thr ? scale : 0.f;
  }
};

Drop make_drop(float p, uint64_t seed) {
  Drop d;
  d.s0 = uint32_t(seed);
  d.s1 = mix32(uint32_t(seed >> 32) ^ 0x5bd1e995u);
  d.on = p > 0.f;
  if (p >= 1.f) {
    d.thr = 0;
    d.scale = 0.f;
  } else {
    const double t = double(p) * 4294967296.0;
    d.thr = t >= 4294967295.0 ? 0xffffffffu : uint32_t(t);
    d.scale = float(1.0 / (1.0 - double(p)));
  }
  return d;
}

struct TrainArgs {
  const float* eh;
  const float* et;
  const float* w1;
  const float* b1;
  const float* w2;
  const int64_t* hist;
  const int64_t* target;
  int64_t b, n;
  int H, D;
  float beta;
  int js;  // history items per slice (blockIdx.y)
  Drop drop;
};

// LDS layout (floats). W1 is kept twice: row-major for the forward A operand (a lane reads 4
// consecutive dims of its hidden row) and transposed for the dx A operand (4 consecutive hidden
// units of its dim row); rows are padded by 4 floats so 16-byte reads of 32 rows hit distinct banks.
template <int DH, int HB>
struct TL {
  static constexpr int D = 2 * DH;
  static constexpr int DW = D < 32 ? 32 : D;  // dims padded to one 32-row MFMA block
  static constexpr int HW = 32 * HB;
  static constexpr int W1P = DW + 4, W1TP = HW + 4, XP = DW + 4, UP = HW + 4;
  static constexpr int O_W1 = 0;
  static constexpr int O_B1 = O_W1 + HW * W1P;
  static constexpr int O_W2 = O_B1 + HW;
  static constexpr int O_H = O_W2 + HW;             // history slice [MAX_JS][D]
  static constexpr int FWD = O_H + MAX_JS * D;
  static constexpr int O_W1T = FWD;                 // backward only from here on
  static constexpr int O_DH = O_W1T + DW * W1TP;    // dh accumulator [MAX_JS][D]
  static constexpr int O_X = O_DH + MAX_JS * D;     // x of the workgroup's rows [TROWS][XP]
  static constexpr int O_U = O_X + TROWS * XP;      // du of the workgroup's rows [TROWS][UP]
  static constexpr int O_BW = O_U + TROWS * UP;     // db1 | dw2 of the workgroup [2][HW]
  static constexpr int BWD = O_BW + 2 * HW;
};

template <int DH, int HB>
__device__ void stage_w(const TrainArgs& a, float* L, int tid, bool transposed) {
  using T = TL<DH, HB>;
  for (int f = tid; f < T::HW * T::DW; f += TTHREADS) {
    const int i = f / T::DW, k = f % T::DW;
    const float v = (i < a.H && k < a.D) ? a.w1[(int64_t)i * a.D + k] : 0.f;
    L[T::O_W1 + i * T::W1P + k] = v;
    if (transposed) L[T::O_W1T + k * T::W1TP + i] = v;
  }
  for (int i = tid; i < T::HW; i += TTHREADS) {
    L[T::O_B1 + i] = i < a.H ? a.b1[i] : 0.f;
    L[T::O_W2 + i] = i < a.H ? a.w2[i] : 0.f;
  }
}

template <int DH, int HB>
__device__ void stage_hist(const TrainArgs& a, float* L, int tid, int64_t j0, int nj) {
  using T = TL<DH, HB>;
  constexpr int D = T::D;
  for (int f = tid; f < nj * (D / 4); f += TTHREADS) {
    const int jj = f / (D / 4), q = f % (D / 4);
    reinterpret_cast<float4*>(L + T::O_H)[f] =
        reinterpret_cast<const float4*>(a.eh + a.hist[j0 + jj] * D)[q];
  }
}

// t_c in K order (kdim) for this lane; zeros for rows past the batch.
template <int DH>
__device__ __forceinline__ void load_target(const TrainArgs& a, int64_t tgt, bool active, int hh,
                                            float (&t)[DH]) {
#pragma unroll
  for (int g = 0; g < DH / 4; ++g) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) v = *reinterpret_cast<const float4*>(a.et + tgt * (2 * DH) + kdim4(g, hh));
    t[4 * g] = v.x;
    t[4 * g + 1] = v.y;
    t[4 * g + 2] = v.z;
    t[4 * g + 3] = v.w;
  }
}

// Forward of one pair for the lane's row: h (K order), x = t (.) h, acc = dropout(b1 + W1 x)
// (post-dropout v), s = h . t and the attention logit a (both joined over the two lane halves).
template <int DH, int HB>
__device__ __forceinline__ void pair_forward(const TrainArgs& ar, const float* L, const float* hrow,
                                             const float (&t)[DH], int lane, uint32_t pair,
                                             float (&h)[DH], float (&x)[DH], floatx16 (&acc)[HB],
                                             float& sdot, float& a) {
  using T = TL<DH, HB>;
  const int hh = lane >> 5, ci = lane & 31;
  float sp = 0.f;
#pragma unroll
  for (int g = 0; g < DH / 4; ++g) {
    const float4 h4 = *reinterpret_cast<const float4*>(hrow + kdim4(g, hh));
    h[4 * g] = h4.x;
    h[4 * g + 1] = h4.y;
    h[4 * g + 2] = h4.z;
    h[4 * g + 3] = h4.w;
  }
#pragma unroll
  for (int s = 0; s < DH; ++s) {
    x[s] = t[s] * h[s];
    sp += x[s];
  }
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[hb][r] = L[T::O_B1 + crow(hb, r, hh)];
    const float* wrow = L + T::O_W1 + (32 * hb + ci) * T::W1P;
#pragma unroll
    for (int g = 0; g < DH / 4; ++g) {
      const float4 w = *reinterpret_cast<const float4*>(wrow + kdim4(g, hh));
      acc[hb] = mfma(w.x, x[4 * g], acc[hb]);
      acc[hb] = mfma(w.y, x[4 * g + 1], acc[hb]);
      acc[hb] = mfma(w.z, x[4 * g + 2], acc[hb]);
      acc[hb] = mfma(w.w, x[4 * g + 3], acc[hb]);
    }
  }
  float ap = 0.f;
  const uint32_t k = ar.drop.on ? ar.drop.key(pair) : 0u;
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = crow(hb, r, hh);
      float v = acc[hb][r];
      if (ar.drop.on) v *= ar.drop.factor(k, i);
      acc[hb][r] = v;
      ap = fmaf(L[T::O_W2 + i], nais_relu(v), ap);
    }
  }
  a = ap + __shfl_xor(ap, 32);
  sdot = sp + __shfl_xor(sp, 32);
}

// Sum of v[] over the 32 lanes of each lane half (a reduce-scatter butterfly: NV-1 + 5-log2(NV)
// shuffles instead of 5 NV). Afterwards lane (ci, hh) holds the total of entry ci >> (5 - log2 NV).
template <int NV, int CNT, int O>
__device__ __forceinline__ void rs_step(float (&v)[NV], int lane) {
  if constexpr (O > 0) {
    if constexpr (CNT > 1) {
      constexpr int HL = CNT / 2;
      const bool up = lane & O;
#pragma unroll
      for (int m = 0; m < HL; ++m) {
        const float send = up ? v[m] : v[m + HL];
        const float keep = up ? v[m + HL] : v[m];
        v[m] = keep + __shfl_xor(send, O);
      }
      rs_step<NV, HL, O / 2>(v, lane);
    } else {
      v[0] += __shfl_xor(v[0], O);
      rs_step<NV, 1, O / 2>(v, lane);
    }
  }
}
template <int NV>
__device__ __forceinline__ float half_reduce_scatter(float (&v)[NV], int lane) {
  rs_step<NV, NV, 16>(v, lane);
  return v[0];
}

template <int NV>
constexpr int log2c() {
  return NV <= 1 ? 0 : 1 + log2c<NV / 2>();
}

// ---------------------------------------------------------------------------------------------
// Forward: grid (ceil(b / 128), ceil(n / js)); per (row, slice) the partial S and N.
// ---------------------------------------------------------------------------------------------
template <int DH, int HB>
__global__ void __launch_bounds__(TTHREADS)
train_forward_kernel(TrainArgs a, float* __restrict__ Sp, float* __restrict__ Np) {
  using T = TL<DH, HB>;
  extern __shared__ float4 lds4[];
  float* L = reinterpret_cast<float*>(lds4);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5;
  const int64_t c = int64_t(blockIdx.x) * TROWS + w * 32 + (lane & 31);
  const int64_t j0 = int64_t(blockIdx.y) * a.js;
  const int nj = (int)(a.n - j0 < a.js ? a.n - j0 : a.js);
  const bool active = c < a.b;
  const int64_t tgt = active ? a.target[c] : -1;
  stage_w<DH, HB>(a, L, tid, false);
  stage_hist<DH, HB>(a, L, tid, j0, nj);
  float t[DH];
  load_target<DH>(a, tgt, active, hh, t);
  __syncthreads();
  float S = 0.f, N = 0.f;
  for (int jj = 0; jj < nj; ++jj) {
    float h[DH], x[DH], sdot, at;
    floatx16 acc[HB];
    pair_forward<DH, HB>(a, L, L + T::O_H + jj * T::D, t, lane, uint32_t(c * a.n + j0 + jj), h, x,
                         acc, sdot, at);
    const float e = expf(at) * (a.hist[j0 + jj] != tgt ? 1.f : 0.f);  // model.py:74-78
    S += e;
    N = fmaf(e, sdot, N);
  }
  if (active && hh == 0) {
    Sp[int64_t(blockIdx.y) * a.b + c] = S;
    Np[int64_t(blockIdx.y) * a.b + c] = N;
  }
}

// S, N over the slices -> logit (model.py:79-89), pred = sigmoid (model.py:55), NaN count.
__global__ void train_finalize_kernel(const float* __restrict__ Sp, const float* __restrict__ Np,
                                      int ns, int64_t b, int64_t n, float beta, float* pred,
                                      float* saved, int32_t* nan_count) {
  const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= b) return;
  float S = 0.f, N = 0.f;
  for (int s = 0; s < ns; ++s) {
    S += Sp[int64_t(s) * b + c];
    N += Np[int64_t(s) * b + c];
  }
  float logit = 0.f;  // empty history: the sum over n is 0
  if (n > 0) logit = N / ((beta == 0.5f) ? sqrtf(S) : powf(S, beta));
  pred[c] = 1.0f / (1.0f + expf(-logit));
  saved[c] = S;
  saved[b + c] = N;
  if (nan_count && logit != logit) atomicAdd(nan_count, 1);
}

// Fused-step variant of the finalize: also the BCELoss of model.py:21 / run.py:104 (mean over the
// b rows, log clamped at -100 as torch does) added into *loss_sum, and dL/dpred of its backward,
// (p - y) / max((1 - p) p, 1e-12) / b. Rows whose prediction is NaN are counted in *bad_rows (the
// reference's BCELoss raises on them); the update kernels then skip the step.
__global__ void train_loss_kernel(const float* __restrict__ Sp, const float* __restrict__ Np,
                                  int ns, int64_t b, int64_t n, float beta,
                                  const float* __restrict__ labels, float* pred, float* saved,
                                  float* gpred, float* loss_sum, int32_t* bad_rows) {
  __shared__ float red[256 / 64];
  const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  float term = 0.f;
  if (c < b) {
    float S = 0.f, N = 0.f;
    for (int s = 0; s < ns; ++s) {
      S += Sp[int64_t(s) * b + c];
      N += Np[int64_t(s) * b + c];
    }
    float logit = 0.f;
    if (n > 0) logit = N / ((beta == 0.5f) ? sqrtf(S) : powf(S, beta));
    const float p = 1.0f / (1.0f + expf(-logit));
    const float y = labels[c];
    pred[c] = p;
    saved[c] = S;
    saved[b + c] = N;
    if (!(p >= 0.f && p <= 1.f)) atomicAdd(bad_rows, 1);
    term = -(y * fmaxf(logf(p), -100.f) + (1.f - y) * fmaxf(logf(1.f - p), -100.f));
    gpred[c] = (p - y) / fmaxf((1.f - p) * p, 1e-12f) / float(b);
  }
  for (int o = 32; o > 0; o >>= 1) term += __shfl_xor(term, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = term;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    atomicAdd(loss_sum, t / float(b));
  }
}

// ---------------------------------------------------------------------------------------------
// Backward: same grid as the forward. Gradients are ADDED into the caller's buffers (fp32
// atomics: the dense embedding grads by POI id, so repeated ids are summed as index_add does).
// ---------------------------------------------------------------------------------------------
template <int DH, int HB>
__global__ void __launch_bounds__(TTHREADS, 1)
train_backward_kernel(TrainArgs a, const float* __restrict__ saved, const float* __restrict__ pred,
                      const float* __restrict__ gpred, float* __restrict__ Wt,
                      float* __restrict__ Ww, float* __restrict__ Wh) {
  TSTART();
  using T = TL<DH, HB>;
  constexpr int D = T::D;
  constexpr int DB = (DH + 15) / 16;             // 32-dim blocks of dx / dW1 columns
  constexpr int NT = HB * DB;                    // 32x32 tiles of dW1
  constexpr int TPW = (NT + TW - 1) / TW;        // tiles per wave
  constexpr int SHD = 5 - log2c<DH>();           // reduce-scatter entry shift (dims)
  constexpr int SHH = 5 - log2c<16 * HB>();      // reduce-scatter entry shift (hidden)
  extern __shared__ float4 lds4[];
  float* L = reinterpret_cast<float*>(lds4);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, ci = lane & 31;
  const int64_t c = int64_t(blockIdx.x) * TROWS + w * 32 + ci;
  const int64_t j0 = int64_t(blockIdx.y) * a.js;
  const int nj = (int)(a.n - j0 < a.js ? a.n - j0 : a.js);
  const bool active = c < a.b;
  const int64_t tgt = active ? a.target[c] : -1;

  stage_w<DH, HB>(a, L, tid, true);
  stage_hist<DH, HB>(a, L, tid, j0, nj);
  for (int f = tid; f < MAX_JS * D; f += TTHREADS) L[T::O_DH + f] = 0.f;
  for (int f = tid; f < 2 * T::HW; f += TTHREADS) L[T::O_BW + f] = 0.f;
  for (int f = tid; f < TROWS * T::XP; f += TTHREADS) L[T::O_X + f] = 0.f;  // dims >= D stay 0
  float t[DH];
  load_target<DH>(a, tgt, active, hh, t);

  // per-row scalars: g = dL/dlogit (sigmoid backward of the reference: grad * (1 - y) * y)
  float gl = 0.f, bns = 0.f;
  if (active) {
    const float p = pred[c], S = saved[c], N = saved[a.b + c];
    const float g = gpred[c] * (1.f - p) * p;
    gl = g / ((a.beta == 0.5f) ? sqrtf(S) : powf(S, a.beta));
    bns = a.beta * N / S;
  }
  const float sc = a.drop.on ? a.drop.scale : 1.f;

  float dt[DH];
#pragma unroll
  for (int s = 0; s < DH; ++s) dt[s] = 0.f;
  float gb1[16 * HB], gw2[16 * HB];
#pragma unroll
  for (int q = 0; q < 16 * HB; ++q) gb1[q] = gw2[q] = 0.f;
  floatx16 gw[TPW];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
    for (int r = 0; r < 16; ++r) gw[tt][r] = 0.f;
  __syncthreads();

  TMARK(0);
  float* xrow = L + T::O_X + (w * 32 + ci) * T::XP;
  float* urow = L + T::O_U + (w * 32 + ci) * T::UP;
  for (int jj = 0; jj < nj; ++jj) {
    float h[DH], x[DH], sdot, at;
    floatx16 acc[HB];
    pair_forward<DH, HB>(a, L, L + T::O_H + jj * D, t, lane, uint32_t(c * a.n + j0 + jj), h, x,
                         acc, sdot, at);
    const float e = expf(at) * (a.hist[j0 + jj] != tgt ? 1.f : 0.f);
    TMARK(1);
    const float ds = gl * e;
    const float da = ds * (sdot - bns);
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = crow(hb, r, hh);
        const float v = acc[hb][r];
        const float wi = L[T::O_W2 + i];
        gw2[hb * 16 + r] = fmaf(da, nais_relu(v), gw2[hb * 16 + r]);
        const float du = v > 0.f ? da * wi * sc : 0.f;
        gb1[hb * 16 + r] += du;
        acc[hb][r] = du;
      }
    }
    // x and du of this row into LDS for the dW1 product (K = the workgroup's rows)
#pragma unroll
    for (int g = 0; g < DH / 4; ++g)
      *reinterpret_cast<float4*>(xrow + kdim4(g, hh)) =
          make_float4(x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]);
#pragma unroll
    for (int hb = 0; hb < HB; ++hb)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(urow + 32 * hb + 8 * g + 4 * hh) =
            make_float4(acc[hb][4 * g], acc[hb][4 * g + 1], acc[hb][4 * g + 2], acc[hb][4 * g + 3]);

    TMARK(2);
    // dx = W1^T du, du taken from the accumulator registers as the B operand
    floatx16 dx[DB];
#pragma unroll
    for (int db = 0; db < DB; ++db) {
#pragma unroll
      for (int r = 0; r < 16; ++r) dx[db][r] = 0.f;
      const float* wt = L + T::O_W1T + (32 * db + ci) * T::W1TP;
#pragma unroll
      for (int hb = 0; hb < HB; ++hb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 wv = *reinterpret_cast<const float4*>(wt + 32 * hb + 8 * g + 4 * hh);
          dx[db] = mfma(wv.x, acc[hb][4 * g], dx[db]);
          dx[db] = mfma(wv.y, acc[hb][4 * g + 1], dx[db]);
          dx[db] = mfma(wv.z, acc[hb][4 * g + 2], dx[db]);
          dx[db] = mfma(wv.w, acc[hb][4 * g + 3], dx[db]);
        }
    }
    float vh[DH];
#pragma unroll
    for (int s = 0; s < DH; ++s) {
      const float r = dx[s >> 4][s & 15] + ds;
      dt[s] = fmaf(r, h[s], dt[s]);
      vh[s] = r * t[s];
    }
    TMARK(3);
    const float hsum = half_reduce_scatter<DH>(vh, lane);
    if ((ci & ((1 << SHD) - 1)) == 0) atomicAdd(&L[T::O_DH + jj * D + kdim(ci >> SHD, hh)], hsum);
    TMARK(4);
    __syncthreads();
    TMARK(5);
    // dW1 tiles: A = du^T rows (hidden), B = x rows (dims), K over the 128 rows
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int tile = w + TW * tt;
      if (tile < NT) {
        const int ib = tile / DB, kb = tile % DB;
        const float* ua = L + T::O_U + 32 * ib + ci;
        const float* xb = L + T::O_X + 32 * kb + ci;
#pragma unroll 8
        for (int kk = 0; kk < TROWS / 2; ++kk) {
          const int row = 2 * kk + hh;
          gw[tt] = mfma(ua[row * T::UP], xb[row * T::XP], gw[tt]);
        }
      }
    }
    TMARK(6);
    __syncthreads();
    TMARK(7);
  }

  // ---- partials of this workgroup (plain stores; train_reduce_kernel sums them):
  //   Wt [slices][b][D] dt per row, Ww [workgroups][H*D + 2H] dW1 | db1 | dw2,
  //   Wh [row blocks][n][D] dh per history item
  const int64_t blk = int64_t(blockIdx.y) * gridDim.x + blockIdx.x;
  const int wsz = a.H * D + 2 * a.H;
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    const int tile = w + TW * tt;
    if (tile < NT) {
      const int ib = tile / DB, kb = tile % DB;
      const int col = 32 * kb + ci;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = crow(ib, r, hh);
        if (row < a.H && col < D) Ww[blk * wsz + row * D + col] = gw[tt][r];
      }
    }
  }
  {
    const float sb = half_reduce_scatter<16 * HB>(gb1, lane);
    const float sw = half_reduce_scatter<16 * HB>(gw2, lane);
    if ((ci & ((1 << SHH) - 1)) == 0) {
      const int m = ci >> SHH;
      const int i = crow(m >> 4, m & 15, hh);
      atomicAdd(&L[T::O_BW + i], sb);
      atomicAdd(&L[T::O_BW + T::HW + i], sw);
    }
  }
  if (active) {
    float* dst = Wt + (int64_t(blockIdx.y) * a.b + c) * D;
#pragma unroll
    for (int g = 0; g < DH / 4; ++g)
      *reinterpret_cast<float4*>(dst + kdim4(g, hh)) =
          make_float4(dt[4 * g], dt[4 * g + 1], dt[4 * g + 2], dt[4 * g + 3]);
  }
  __syncthreads();
  for (int i = tid; i < a.H; i += TTHREADS) {
    Ww[blk * wsz + a.H * D + i] = L[T::O_BW + i];
    Ww[blk * wsz + a.H * D + a.H + i] = L[T::O_BW + T::HW + i];
  }
  for (int f = tid; f < nj * D; f += TTHREADS)
    Wh[(int64_t(blockIdx.x) * a.n + j0) * D + f] = L[T::O_DH + f];
  TMARK(8);
  TFLUSH();
}

constexpr int REDUCE_KS = 16;

// Sums the backward partials into the caller's gradients (+=): dW1 | db1 | dw2 over workgroups,
// dt over slices scattered to embed_target rows, dh over row blocks scattered to embed_history
// rows (atomics only for the two scatters, where POI ids may repeat).
__global__ void train_reduce_kernel(const float* __restrict__ Wt, const float* __restrict__ Ww,
                                    const float* __restrict__ Wh, int64_t b, int64_t n, int D,
                                    int H, int ns, int rb, const int64_t* __restrict__ hist,
                                    const int64_t* __restrict__ target, float* g_eh, float* g_et,
                                    float* g_w1, float* g_b1, float* g_w2,
                                    const int32_t* __restrict__ bad_rows) {
  if (bad_rows && *bad_rows) return;  // fused step on a NaN batch: no update (see train_loss)
  const int64_t wsz = int64_t(H) * D + 2 * H;
  const int64_t nblk = int64_t(ns) * rb;
  const int64_t nw = wsz * REDUCE_KS, nt = b * D, nh = n * D;
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e < nw) {  // REDUCE_KS threads per weight, each over every REDUCE_KS-th workgroup
    const int64_t el = e % wsz, part = e / wsz;
    float sum = 0.f;
#pragma unroll 4
    for (int64_t k = part; k < nblk; k += REDUCE_KS) sum += Ww[k * wsz + el];
    float* dst = el < int64_t(H) * D ? g_w1 + el
               : el < int64_t(H) * D + H ? g_b1 + (el - int64_t(H) * D)
                                         : g_w2 + (el - int64_t(H) * D - H);
    unsafeAtomicAdd(dst, sum);
  } else if (e < nw + nt) {
    const int64_t f = e - nw, c = f / D, d = f % D;
    float sum = 0.f;
#pragma unroll 4
    for (int k = 0; k < ns; ++k) sum += Wt[(int64_t(k) * b + c) * D + d];
    unsafeAtomicAdd(&g_et[target[c] * D + d], sum);
  } else if (e < nw + nt + nh) {
    const int64_t f = e - nw - nt, j = f / D, d = f % D;
    float sum = 0.f;
#pragma unroll 4
    for (int k = 0; k < rb; ++k) sum += Wh[(int64_t(k) * n + j) * D + d];
    unsafeAtomicAdd(&g_eh[hist[j] * D + d], sum);
  }
}

__global__ void dropout_mask_kernel(Drop d, int64_t b, int64_t n, int H, uint8_t* out) {
  const int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= b * n * H) return;
  const int i = int(idx % H);
  const int64_t pair = idx / H;
  out[idx] = d.on ? (d.factor(d.key(uint32_t(pair)), i) != 0.f) : 1;
}

// torch.optim.Adagrad (run.py:89) update of one tensor:
//   g += wd p ; state += g g ; p -= clr g / (sqrt(state) + eps)
__global__ void adagrad_kernel(float* __restrict__ p, float* __restrict__ st,
                               const float* __restrict__ g, int64_t numel, float clr, float wd,
                               float eps) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < numel;
       i += int64_t(gridDim.x) * blockDim.x) {
    float gi = g[i];
    const float pi = p[i];
    if (wd != 0.f) gi = gi + wd * pi;
    const float si = st[i] + gi * gi;
    st[i] = si;
    p[i] = pi + (-clr) * (gi / (sqrtf(si) + eps));
  }
}

// The same update restricted to `rows` of a [*, dim] tensor. With weight_decay 0 a row whose
// gradient is zero is left bit-identical by the dense update (state += 0, p -= 0), so this equals
// the dense step when `rows` covers every row with a nonzero gradient. An entry equal to the one
// before it is skipped, so a sorted list with repeats (no device->host sync to dedup) is fine.
__global__ void adagrad_rows_kernel(float* __restrict__ p, float* __restrict__ st,
                                    const float* __restrict__ g, int dim,
                                    const int64_t* __restrict__ rows, int64_t nrows, float clr,
                                    float eps) {
  const int64_t total = nrows * dim;
  for (int64_t f = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; f < total;
       f += int64_t(gridDim.x) * blockDim.x) {
    const int64_t k = f / dim;
    if (k > 0 && rows[k] == rows[k - 1]) continue;
    const int64_t i = rows[k] * dim + f % dim;
    const float gi = g[i];
    const float si = st[i] + gi * gi;
    st[i] = si;
    p[i] = p[i] + (-clr) * (gi / (sqrtf(si) + eps));
  }
}

// Adagrad of the fused step, applied straight from the zero-maintained gradient scratch (which it
// leaves zero again): the small tensors element-wise; the embedding tables row by row for the rows
// the batch touched (history + targets; with weight_decay 0 the other rows' dense update is the
// identity). A row listed twice is claimed once per step through `stamp` (atomicExch of the step
// number), so it is updated once, with its summed gradient. One wave per row, lanes over dims.
struct StepOpt {
  float* p_eh;
  float* p_et;
  float* p_small[3];  // w1, b1, w2
  float* s_eh;
  float* s_et;
  float* s_small[3];
  float* g_eh;
  float* g_et;
  float* g_small;  // [H*D | H | H]
  int32_t* st_eh;
  int32_t* st_et;
  float clr, wd, eps;
  int32_t tag;
};

__device__ __forceinline__ void adagrad_elem(float* p, float* st, float* g, float clr, float wd,
                                             float eps) {
  float gi = *g;
  const float pi = *p;
  if (wd != 0.f) gi = gi + wd * pi;
  const float si = *st + gi * gi;
  *st = si;
  *p = pi + (-clr) * (gi / (sqrtf(si) + eps));
  *g = 0.f;
}

// DIN = attn_layer1's input width (the w1 block of g_small is H x DIN), D = the embedding rows' width
__global__ void step_adagrad_kernel(StepOpt o, int H, int DIN, int D, const int64_t* __restrict__ hist,
                                    int64_t n, const int64_t* __restrict__ target, int64_t b,
                                    int64_t dense_rows, const int32_t* __restrict__ bad_rows) {
  if (*bad_rows) return;
  const int64_t wsz = int64_t(H) * DIN + 2 * H;
  const int64_t nsmall_blocks = (wsz + 255) / 256;
  const int64_t bx = blockIdx.x;
  if (bx < nsmall_blocks) {
    const int64_t e = bx * 256 + threadIdx.x;
    if (e < wsz) {
      const int k = e < int64_t(H) * DIN ? 0 : (e < int64_t(H) * DIN + H ? 1 : 2);
      const int64_t off = k == 0 ? e : (k == 1 ? e - int64_t(H) * DIN : e - int64_t(H) * DIN - H);
      adagrad_elem(o.p_small[k] + off, o.s_small[k] + off, o.g_small + e, o.clr, o.wd, o.eps);
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t item = (bx - nsmall_blocks) * 4 + (threadIdx.x >> 6);
  if (dense_rows > 0) {  // weight_decay != 0: every row of both tables changes
    if (item >= 2 * dense_rows) return;
    const bool tgt = item >= dense_rows;
    const int64_t row = tgt ? item - dense_rows : item;
    for (int d = lane; d < D; d += 64) {
      const int64_t i = row * D + d;
      if (tgt) adagrad_elem(o.p_et + i, o.s_et + i, o.g_et + i, o.clr, o.wd, o.eps);
      else adagrad_elem(o.p_eh + i, o.s_eh + i, o.g_eh + i, o.clr, o.wd, o.eps);
    }
    return;
  }
  if (item >= n + b) return;
  const bool tgt = item >= n;
  const int64_t row = tgt ? target[item - n] : hist[item];
  int claimed = 0;
  if (lane == 0) claimed = atomicExch(tgt ? o.st_et + row : o.st_eh + row, o.tag) != o.tag;
  claimed = __shfl(claimed, 0);
  if (claimed) {
    for (int d = lane; d < D; d += 64) {
      const int64_t i = row * D + d;
      if (tgt) adagrad_elem(o.p_et + i, o.s_et + i, o.g_et + i, o.clr, 0.f, o.eps);
      else adagrad_elem(o.p_eh + i, o.s_eh + i, o.g_eh + i, o.clr, 0.f, o.eps);
    }
  }
}

// Adagrad of a whole small tensor from its zero-maintained gradient scratch (the fused step of the
// region variants: embed_region, every row -- the region ids of a batch are few, and a row whose
// gradient is 0 is left bit-identical with weight_decay 0 -- and dist_layer's weight / bias).
__global__ void step_adagrad_dense_kernel(float* p, float* st, float* g, int64_t numel, float clr,
                                          float wd, float eps, const int32_t* __restrict__ bad_rows) {
  if (*bad_rows) return;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < numel;
       e += int64_t(gridDim.x) * blockDim.x)
    adagrad_elem(p + e, st + e, g + e, clr, wd, eps);
}

// ---------------------------------------------------------------------------------------------
// Device-side get_NAIS_batch (batches.py:24-50) for one user: history = the
// user's positives in a random order, rows [pos_i, neg_i1 .. neg_i,ng], labels 1 / 0. Negatives
// are the first n*ng members, in a pseudo-random order of [0, P), that are not positives: a
// uniformly random distinct subset of the complement, as the reference's shuffle-and-slice --
// the same distribution, not Python's `random` stream. The orders come from a seeded Feistel
// permutation of [0, 4^h) walked down to [0, m) (cycle walking), so no sort is needed.
// ---------------------------------------------------------------------------------------------
// 8-round Feistel network on [0, 2^(2*hb)) keyed by the seed (round function: murmur finaliser;
// 8 rounds: 4 leave a visible bias on domains of a few elements)
__device__ __forceinline__ uint32_t feistel(uint32_t x, int hb, uint32_t s) {
  const uint32_t mh = (1u << hb) - 1u;
  uint32_t L = x >> hb, R = x & mh;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint32_t f = mix32(R ^ (s + uint32_t(r) * 0x9e3779b9u)) & mh;
    const uint32_t t = L ^ f;
    L = R;
    R = t;
  }
  return (L << hb) | R;
}

// bijection of [0, m): the Feistel permutation of [0, 2^(2 hb)) >= m, walked until it lands < m
__device__ __forceinline__ uint32_t permute(uint32_t i, uint32_t m, int hb, uint32_t s) {
  do {
    i = feistel(i, hb, s);
  } while (i >= m);
  return i;
}

// half the bits of the smallest power of two >= m (m >= 2), rounded up
__device__ __forceinline__ int half_bits(uint32_t m) {
  const int k = 32 - __clz(m - 1);
  return (k + 1) >> 1;
}

constexpr int BATCH_THREADS = 1024;

__global__ void __launch_bounds__(BATCH_THREADS)
make_batch_kernel(const int64_t* __restrict__ indptr, const int64_t* __restrict__ indices,
                  int64_t user, int64_t n, int64_t P, int ng, uint32_t s0, uint32_t s1,
                  int64_t* __restrict__ hist, int64_t* __restrict__ target,
                  float* __restrict__ labels, int32_t* __restrict__ err) {
  __shared__ int32_t scan[BATCH_THREADS / 64];
  __shared__ int64_t base;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t start = indptr[user];
  if (tid == 0 && err && indptr[user + 1] - start != n) *err = 1;
  const int64_t* row = indices + start;
  const uint32_t mn = uint32_t(n), mP = uint32_t(P);
  const int hn = mn > 1 ? half_bits(mn) : 0, hP = mP > 1 ? half_bits(mP) : 0;
  for (int64_t i = tid; i < n; i += BATCH_THREADS) {
    const int64_t v = row[mn > 1 ? permute(uint32_t(i), mn, hn, s0) : 0];
    hist[i] = v;
    target[i * (1 + ng)] = v;
    labels[i * (1 + ng)] = 1.f;
  }
  if (tid == 0) base = 0;
  __syncthreads();
  const int64_t want = n * ng;
  for (int64_t k0 = 0; k0 < n * (ng + 1); k0 += BATCH_THREADS) {
    const int64_t k = k0 + tid;
    int64_t cand = -1;
    if (k < n * (ng + 1)) {
      cand = mP > 1 ? permute(uint32_t(k), mP, hP, s1) : 0;
      int64_t lo = 0, hi = n;  // binary search in the sorted CSR row
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (row[mid] < cand) lo = mid + 1;
        else hi = mid;
      }
      if (lo < n && row[lo] == cand) cand = -1;
    }
    const bool acc = cand >= 0;
    const unsigned long long bal = __ballot(acc);
    const int before = __popcll(bal & ((1ull << lane) - 1));
    if (lane == 0) scan[w] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int q = 0; q < BATCH_THREADS / 64; ++q) {
      if (q < w) off += scan[q];
      tot += scan[q];
    }
    const int64_t pos = base + off + before;
    if (acc && pos < want) {
      const int64_t r = pos / ng, q = pos % ng;
      target[r * (1 + ng) + 1 + q] = cand;
      labels[r * (1 + ng) + 1 + q] = 0.f;
    }
    __syncthreads();
    if (tid == 0) base += tot;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// General training kernels: every NAIS variant (basic, region, region_distance; model.py:8-304)
// at embed_dim <= 128 (even), hidden <= 128 -- the dims the fused MFMA kernels above do not cover
// (run.py's defaults are factor_num = hidden_dim = 128) and the region variants' training drivers
// (run.py:153-200, 222-262). Same math, same dropout hash, same S / N partials + finalize.
//   full history row hf_j = [embed_history[h_j] | embed_region[hreg_j]]   (region variants)
//   full target row  tf   = [embed_target[c]    | embed_region[treg_c]]
//   x = hf_j (.) tf [| sigmoid(dist_layer(100 * latlon_cj))]   (region_distance, model.py:265-267)
// One wave per batch row (GW rows per workgroup), the slice's items in turn. W1^T sits in LDS with
// an odd row pitch (H + 1), so the forward (lanes over hidden units) and dx (lanes over dims) both
// read it conflict-free; x and du are broadcast with readlane in uniform loops. The backward
// accumulates dW1 / db1 / dw2 / d(dist_layer) and the slice's history-row grads in LDS (ds_add)
// and adds them to the caller's gradients with global atomics; target-row grads go straight from
// registers.
// ---------------------------------------------------------------------------------------------
constexpr int GW = 12;   // rows (waves) per workgroup: 3 waves per SIMD (153-167 VGPRs); A/B vs 8:
                         // step 0.567 -> 0.530 ms at D = H = 128
constexpr int G_MAX_D = 128, G_MAX_H = 128, G_MAX_DIN = G_MAX_D + 2;

struct GArgs {
  const float *eh, *et, *er, *w1, *b1, *w2, *dw, *db;
  const int64_t *hist, *target, *hreg, *treg;
  const float* ll;
  int64_t ll_ld;
  int64_t b, n;
  int D, IDIM, RDIM, H, DIN, variant;
  float beta, dscale;
  int js;
  Drop drop;
  // fused step only (nais_train_step): the forward's post-dropout u (the wave's accumulator
  // registers), s = h . t and the attention logit of every pair, read back by the backward instead
  // of recomputing them (the third of its MFMA work); NULL = recompute
  float* ucache;
};

struct GGrads {
  float *eh, *et, *er, *w1, *b1, *w2, *dw, *db;
};

__device__ __forceinline__ float rl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// u cache record of one (slice, batch row): HB * 16 accumulator values + s + a logit, 64 lanes
// each, in the forward's order (unit un = slice * row tiles + tile, wave w: sl * tiles * GW + c),
// so a backward with another rows-per-workgroup split finds the same records
__device__ __forceinline__ float* ucache_rec(const GArgs& a, int hb_count, int64_t sl, int64_t c) {
  const int64_t nrt = (a.b + GW - 1) / GW;
  return a.ucache + ((sl * nrt * GW + c) * int64_t(hb_count * 16 + 2)) * 64;
}
size_t ucache_bytes(int H, int64_t b, int64_t n) {
  const int64_t units = ((b + GW - 1) / GW) * ((n + 31) / 32);
  return size_t(units * GW * int64_t(((H + 31) / 32) * 16 + 2) * 64) * sizeof(float);
}
constexpr size_t UCACHE_MAX_BYTES = size_t(1) << 30;   // above: the backward recomputes u
constexpr bool UCACHE_NT = true;   // non-temporal u-cache stores / loads (A/B vs default: 0.512 vs 0.516 ms per step)
__device__ __forceinline__ void uc_store(float v, float* p) {
  if (UCACHE_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ float uc_load(const float* p) {
  if (UCACHE_NT) return __builtin_nontemporal_load(p);
  return *p;
}

// The backward's global atomics at config 3, D = H = 128 (timing-only builds without them,
// profiles/r5/train_bwd/r5diag): dW1 0.033 ms, history-row grads 0.022 ms of the 0.427 ms.

// The general backward runs one unit per workgroup (a persistent form keeping W1 staged across
// units spills at D = H = 128; its code path stays for the shapes that may use it).
constexpr bool GM_BWD_PERSIST = false;

// The LDS base as an opaque per-iteration value: inside the persistent unit loops, reads of the
// loop-invariant W1 image would otherwise be hoisted out of the loop into (spilled) registers.
__device__ __forceinline__ float* opaque_lds(float* L) {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return L + z;
}

// element d of the full history / target row
__device__ __forceinline__ float hfull(const GArgs& a, int64_t j, int d) {
  if (d >= a.D) return 0.f;
  if (d < a.IDIM) return a.eh[a.hist[j] * a.IDIM + d];
  return a.er[a.hreg[j] * a.RDIM + (d - a.IDIM)];
}
__device__ __forceinline__ float tfull(const GArgs& a, int64_t c, int d) {
  if (d >= a.D) return 0.f;
  if (d < a.IDIM) return a.et[a.target[c] * a.IDIM + d];
  return a.er[a.treg[c] * a.RDIM + (d - a.IDIM)];
}

// Shape of one general-kernel instantiation: compile-time D / H / extra input dims where the
// template fixes them (the reference defaults, D = H = 128: every loop below then has a constant
// trip count, is unrolled and its LDS operand reads are scheduled ahead of the MFMAs), the
// runtime GArgs values otherwise (DC = 0).
struct GS {
  int D, H, DIN;
};
template <int DC, int HC, int XC>
__device__ __forceinline__ GS make_gs(const GArgs& a) {
  if constexpr (DC > 0) return GS{DC, HC, DC + XC};
  else return GS{a.D, a.H, a.DIN};
}

// LDS image of the general kernels (floats). Hidden rows are padded to HB*32 (zeros), x to
// DINP = DIN rounded up to even (K-steps of 2); pitches are odd so that every MFMA operand read
// (lanes over rows at a fixed column, or over columns at a fixed row) is bank-conflict-free.
struct GL {
  int HB, HP32, DINP, Q;        // hidden blocks, padded hidden, padded din, W1 pitch (DINP + 1)
  int HD;                       // history-slice row pitch (D + 1)
  int DBX, XP, UP;              // x blocks of the dW1 tiles (ceil(DIN/32)), stage pitches
  int o_w1, o_b1, o_w2, o_hs, o_ts, o_fs, fwd;
  int o_gh, o_su, o_sx, o_gb, o_gw, o_gd, bwd;
  __host__ __device__ GL(int D, int H, int DIN, int gw = GW) {
    HB = (H + 31) / 32;
    HP32 = HB * 32;
    DINP = (DIN + 1) & ~1;
    Q = DINP + 1;
    HD = D + 1;
    DBX = (DIN + 31) / 32;
    XP = DBX * 32 + 1;
    UP = HP32 + 1;
    o_w1 = 0;
    o_b1 = o_w1 + HP32 * Q;
    o_w2 = o_b1 + HP32;
    o_hs = o_w2 + HP32;                 // [32][HD] full history rows of the slice
    o_ts = o_hs + 32 * HD;              // [GW][D]  full target rows of the workgroup
    o_fs = o_ts + gw * D;               // [GW][32][4] f0, f1, 100 lat, 100 lng (region_distance)
    fwd = o_fs + gw * 32 * 4;
    o_gh = fwd;                         // [32][HD] history-row grads of the slice (odd pitch:
                                        //          the 32 lanes' items hit distinct banks)
    o_su = o_gh + 32 * HD;              // [2][32][UP] du^T stages (one wave's pairs each; double
                                        //             buffered: the next wave stages while the
                                        //             current one's are consumed)
    o_sx = o_su + 32 * UP;              // the second du stage
    o_gb = o_sx + 32 * UP;              // [HP32] db1
    o_gw = o_gb + HP32;                 // [HP32] dw2
    o_gd = o_gw + HP32;                 // [8]    dist_layer dw | db
    bwd = o_gd + 8;
  }
};

// stage W1 (row-major, pitch Q, zero padded), b1, w2 -- once per (persistent) workgroup
template <int GWT = GW>
__device__ __forceinline__ void gm_stage_w(const GArgs& a, const GS& s, const GL& g, float* L, int tid) {
  constexpr int NT = GWT * 64;
  if (s.DIN % 4 == 0 && s.H == g.HP32 && (reinterpret_cast<uintptr_t>(a.w1) & 15) == 0) {
    // 16-byte global reads (the D = H = 128 shape: 4,096 float4), then the zero pad columns
    const int R4 = s.DIN / 4;
    for (int f = tid; f < s.H * R4; f += NT) {
      const int i = f / R4, k = 4 * (f % R4);
      const float4 v = reinterpret_cast<const float4*>(a.w1)[f];
      float* o = L + g.o_w1 + i * g.Q + k;
      o[0] = v.x;
      o[1] = v.y;
      o[2] = v.z;
      o[3] = v.w;
    }
    const int PC = g.Q - s.DIN;
    for (int f = tid; f < g.HP32 * PC; f += NT) L[g.o_w1 + (f / PC) * g.Q + s.DIN + f % PC] = 0.f;
  } else {
    for (int f = tid; f < g.HP32 * g.Q; f += NT) {
      const int i = f / g.Q, k = f % g.Q;
      L[g.o_w1 + f] = (i < s.H && k < s.DIN) ? a.w1[int64_t(i) * s.DIN + k] : 0.f;
    }
  }
  for (int i = tid; i < g.HP32; i += NT) {
    L[g.o_b1 + i] = i < s.H ? a.b1[i] : 0.f;
    L[g.o_w2 + i] = i < s.H ? a.w2[i] : 0.f;
  }
}

// one work unit's operands: the slice's full history rows, the row tile's full target rows
template <int GWT = GW>
__device__ __forceinline__ void gm_stage(const GArgs& a, const GS& s, const GL& g, float* L, int tid,
                                         int64_t c0, int64_t j0, int nj) {
  constexpr int NT = GWT * 64;
  for (int f = tid; f < 32 * g.HD; f += NT) {
    const int n = f / g.HD, d = f % g.HD;
    L[g.o_hs + f] = (n < nj && d < s.D) ? hfull(a, j0 + n, d) : 0.f;
  }
  for (int f = tid; f < GWT * s.D; f += NT) {
    const int w = f / s.D, d = f % s.D;
    const int64_t c = c0 + w;
    L[g.o_ts + f] = c < a.b ? tfull(a, c, d) : 0.f;
  }
  if (s.DIN > s.D) {
    for (int f = tid; f < GWT * 32; f += NT) {
      const int w = f / 32, n = f % 32;
      const int64_t c = c0 + w;
      float f0 = 0.f, f1 = 0.f, l0 = 0.f, l1 = 0.f;
      if (c < a.b && n < nj) {
        const float* ll = a.ll + c * a.ll_ld + 2 * (j0 + n);
        l0 = ll[0] * a.dscale;
        l1 = ll[1] * a.dscale;
        // sigmoid(dist_layer(100 ll)), model.py:265, in the scorer's operation order
        f0 = 1.0f / (1.0f + expf(-(l0 * a.dw[0] + l1 * a.dw[1] + a.db[0])));
        f1 = 1.0f / (1.0f + expf(-(l0 * a.dw[2] + l1 * a.dw[3] + a.db[1])));
      }
      float* o = L + g.o_fs + f * 4;
      o[0] = f0;
      o[1] = f1;
      o[2] = l0;
      o[3] = l1;
    }
  }
}

// x[k][n] of the wave's row and item n (0 past din)
__device__ __forceinline__ float gm_x(const GS& s, const GL& g, const float* L, int w, int n, int k) {
  if (k < s.D) return L[g.o_hs + n * g.HD + k] * L[g.o_ts + w * s.D + k];
  if (k < s.DIN) return L[g.o_fs + (w * 32 + n) * 4 + (k - s.D)];
  return 0.f;
}

// Forward of the wave's 32 pairs (row c, items j0 + n): acc[hb] = dropout(b1 + W1 x) in the
// 32x32 C layout (rows = hidden units, columns = pairs), the pair's h . t and attention logit.
template <int HBM>
__device__ __forceinline__ void gm_pair_forward(const GArgs& a, const GS& s, const GL& g, const float* L, int w,
                                                int lane, int64_t c, int64_t j0, floatx16 (&acc)[HBM],
                                                float& sdot, float& alogit) {
  const int hh = lane >> 5, n = lane & 31;
#pragma unroll
  for (int hb = 0; hb < HBM; ++hb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[hb][r] = hb < g.HB ? L[g.o_b1 + crow(hb, r, hh)] : 0.f;
  float sp = 0.f;
#pragma unroll
  for (int t = 0; t < g.DINP / 2; ++t) {
    const int k = 2 * t + hh;
    const float x = gm_x(s, g, L, w, n, k);
    if (k < s.D) sp += x;
#pragma unroll
    for (int hb = 0; hb < HBM; ++hb)
      if (hb < g.HB) acc[hb] = mfma(L[g.o_w1 + (32 * hb + n) * g.Q + k], x, acc[hb]);
  }
  sdot = sp + __shfl_xor(sp, 32);
  float ap = 0.f;
  const uint32_t key = a.drop.on ? a.drop.key(uint32_t(c * a.n + j0 + n)) : 0u;
#pragma unroll
  for (int hb = 0; hb < HBM; ++hb) {
    if (hb >= g.HB) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = crow(hb, r, hh);
      float v = acc[hb][r];
      if (a.drop.on) v *= a.drop.factor(key, i);
      acc[hb][r] = v;
      ap = fmaf(L[g.o_w2 + i], nais_relu(v), ap);
    }
  }
  alogit = ap + __shfl_xor(ap, 32);
}

// sum over the 32 lanes of one half (both halves get it)
__device__ __forceinline__ float half_sum(float v) {
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// GWT rows (waves) per workgroup, slices sl0, sl0 + 1, ... (g_forward's split launch, as the
// backward's)
template <int HBM, int DC = 0, int HC = 0, int XC = 0, int GWT = GW>
__global__ void __launch_bounds__(GWT * 64)
gm_forward_kernel(GArgs a, float* __restrict__ Sp, float* __restrict__ Np, int32_t sl0, int32_t trows) {
  extern __shared__ float4 glds4[];
  float* Lb = reinterpret_cast<float*>(glds4);
  const GS s = make_gs<DC, HC, XC>(a);
  const GL g(s.D, s.H, s.DIN, GWT);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 31;
  // persistent: W1 staged once, then work units (row tile of GWT rows, slice of 32 items), row
  // tile fastest, strided over the grid. trows > 0: the short last slice's units are tiles of
  // trows rows (waves >= trows idle in them), so they spread over more workgroups' last round
  gm_stage_w<GWT>(a, s, g, Lb, tid);
  const int64_t nrt = (a.b + GWT - 1) / GWT, nsl = (a.n + 31) / 32 - sl0;
  const int64_t nrt_t = trows > 0 ? (a.b + trows - 1) / trows : 0;
  const int64_t ufull = trows > 0 ? nrt * (nsl - 1) : nrt * nsl;
  const int64_t units = ufull + (trows > 0 ? nrt_t : 0);
  for (int64_t un = blockIdx.x; un < units; un += gridDim.x) {
    const bool tu = un >= ufull;
    const int64_t sl = tu ? sl0 + nsl - 1 : sl0 + un / nrt;
    const int64_t c0 = tu ? (un - ufull) * trows : (un % nrt) * GWT;
    const int64_t c = (tu && w >= trows) ? a.b : c0 + w;   // idle waves: past the last row
    const int64_t j0 = sl * 32;
    const int nj = (int)(a.n - j0 < 32 ? a.n - j0 : 32);
    __syncthreads();   // the previous unit's operand reads are done
    float* L = opaque_lds(Lb);
    gm_stage<GWT>(a, s, g, L, tid, c0, j0, nj);
    __syncthreads();
    if (c < a.b) {
      floatx16 acc[HBM];
      float sdot, at;
      gm_pair_forward<HBM>(a, s, g, L, w, lane, c, j0, acc, sdot, at);
      if (a.ucache) {
        float* rec = ucache_rec(a, g.HB, sl, c) + lane;
#pragma unroll
        for (int hb = 0; hb < HBM; ++hb)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (hb < g.HB) uc_store(acc[hb][r], rec + (hb * 16 + r) * 64);
        uc_store(sdot, rec + (g.HB * 16) * 64);
        uc_store(at, rec + (g.HB * 16 + 1) * 64);
      }
      float e = 0.f;
      if (n < nj) e = expf(at) * (a.hist[j0 + n] != a.target[c] ? 1.f : 0.f);   // model.py:74-78
      const float S = half_sum(e), N = half_sum(e * sdot);
      if (lane == 0) {
        Sp[sl * a.b + c] = S;
        Np[sl * a.b + c] = N;
      }
    }
  }
}

// GWT rows (waves) per workgroup; the units cover slices sl0, sl0 + 1, ... (g_backward's split
// launch: GW rows over the full 32-item slices, GW_TAIL rows over a short last slice)
template <int HBM, int DC = 0, int HC = 0, int XC = 0, int GWT = GW>
__global__ void __launch_bounds__(GWT * 64, 1)
gm_backward_kernel(GArgs a, const float* __restrict__ saved, const float* __restrict__ pred,
                   const float* __restrict__ gpred, GGrads gr, const int32_t* __restrict__ bad_rows,
                   int32_t sl0) {
  if (bad_rows && *bad_rows) return;   // fused step on a NaN batch: no update (see train_loss)
  extern __shared__ float4 glds4[];
  float* Lb = reinterpret_cast<float*>(glds4);
  const GS s = make_gs<DC, HC, XC>(a);
  const GL g(s.D, s.H, s.DIN, GWT);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 31, hh = lane >> 5;
  // persistent: W1 staged once and db1 / dw2 / dist_layer grads kept in LDS across all of the
  // workgroup's units (row tile of GWT rows, slice of 32 items), flushed once; the dW1 tiles and the
  // history-row grads are flushed per unit (registers: the dW1 tiles are live in its last phase only)
  TSTART();   // timing builds: phases 0 W1 + unit staging, 1 u cache, 2 du / db1 / dw2, 3 dx MFMA,
             // 4 history / target row grads, 5 dW1 rounds, 6 dW1 atomics, 7 history-row atomics, 8 flush
  gm_stage_w<GWT>(a, s, g, Lb, tid);
  for (int f = tid; f < 2 * g.HP32 + 8; f += GWT * 64) Lb[g.o_gb + f] = 0.f;
  const int ntile = g.HB * g.DBX;
  const int64_t nrt = (a.b + GWT - 1) / GWT, units = nrt * ((a.n + 31) / 32 - sl0);
  // one unit: the loop body of the persistent form (a lambda, so that the one-unit-per-workgroup
  // launch below carries no loop state -- the persistent loop spills the D = H = 128 backward)
  auto unit = [&](int64_t un) {
    // (slice-minor units, so that the units running at the same time add their history-row grads
    // to different rows: backward 0.428 vs 0.428 ms; dW1 atomics into 4 / 16 replicas plus a reduce:
    // 0.43-0.44 ms -- not kept, profiles/r5/train_bwd)
    const int64_t sl = sl0 + un / nrt, c0 = (un % nrt) * GWT, c = c0 + w;
    const bool live = c < a.b;
    const int64_t j0 = sl * 32;
    const int nj = (int)(a.n - j0 < 32 ? a.n - j0 : 32);
    __syncthreads();   // the previous unit's operand reads and grad flush are done
    float* L = opaque_lds(Lb);
    gm_stage<GWT>(a, s, g, L, tid, c0, j0, nj);
    for (int f = tid; f < 32 * g.HD; f += GWT * 64) L[g.o_gh + f] = 0.f;
    __syncthreads();
    TMARK(0);

    // ---- recompute the forward, then du in place (C layout)
    floatx16 acc[HBM];
    float sdot = 0.f, at = 0.f;
    const int64_t tgt = live ? a.target[c] : -1;
    float e = 0.f;
    if (live && a.ucache) {   // the fused step's forward left u, s and the logit behind
      const float* rec = ucache_rec(a, g.HB, sl, c) + lane;
#pragma unroll
      for (int hb = 0; hb < HBM; ++hb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          acc[hb][r] = hb < g.HB ? uc_load(rec + (hb * 16 + r) * 64) : 0.f;
      sdot = uc_load(rec + (g.HB * 16) * 64);
      at = uc_load(rec + (g.HB * 16 + 1) * 64);
      if (n < nj) e = expf(at) * (a.hist[j0 + n] != tgt ? 1.f : 0.f);
    } else if (live) {
      gm_pair_forward<HBM>(a, s, g, L, w, lane, c, j0, acc, sdot, at);
      if (n < nj) e = expf(at) * (a.hist[j0 + n] != tgt ? 1.f : 0.f);
    } else {
  #pragma unroll
      for (int hb = 0; hb < HBM; ++hb)
  #pragma unroll
        for (int r = 0; r < 16; ++r) acc[hb][r] = 0.f;
    }
    float ds = 0.f, da = 0.f;
    if (live) {
      const float S = saved[c], N = saved[a.b + c], pc = pred[c];
      const float gl = gpred[c] * pc * (1.f - pc);                // dL/dlogit (sigmoid)
      const float Sb = (a.beta == 0.5f) ? sqrtf(S) : powf(S, a.beta);
      ds = gl / Sb * e;                                           // dlogit / ds_cj
      da = ds * (sdot - a.beta * N / S);                          // dlogit / da_cj
    }
    TMARK(1);
    const float kscale = a.drop.on ? a.drop.scale : 1.f;
    // du in place; db1 / dw2 as sums over the 32 pairs of each half (reduce-scatter), LDS atomics
  #pragma unroll
    for (int hb = 0; hb < HBM; ++hb) {
      if (hb >= g.HB) continue;
      float vb[16], vz[16];
  #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = crow(hb, r, hh);
        const float v = acc[hb][r];
        // ReLU + dropout backward: v = u * m > 0 only where the unit was kept (m = scale), so the
        // mask needs no second hash here -- bit-identical to da * w2 * m
        const float du = v > 0.f ? da * L[g.o_w2 + i] * kscale : 0.f;
        acc[hb][r] = du;
        vb[r] = du;
        vz[r] = da * nais_relu(v);
      }
      const float tb = half_reduce_scatter<16>(vb, lane);
      const float tz = half_reduce_scatter<16>(vz, lane);
      if ((n & 1) == 0 && live) {
        const int i = crow(hb, n >> 1, hh);
        atomicAdd(&L[g.o_gb + i], tb);
        atomicAdd(&L[g.o_gw + i], tz);
      }
    }
    TMARK(2);
    // ---- dx = W1^T du (K-step (hb, r) = hidden unit crow(hb, r, hh): du straight from acc)
    constexpr int DBM = 4;
    floatx16 dx[DBM];
    const int DB = (s.D + 31) / 32;
  #pragma unroll
    for (int q = 0; q < DBM; ++q)
  #pragma unroll
      for (int r = 0; r < 16; ++r) dx[q][r] = 0.f;
    float df0 = 0.f, df1 = 0.f;
  #pragma unroll
    for (int hb = 0; hb < HBM; ++hb) {
      if (hb >= g.HB) continue;
  #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = crow(hb, r, hh);
        const float du = acc[hb][r];
        const float* wrow = L + g.o_w1 + i * g.Q;
  #pragma unroll
        for (int q = 0; q < DBM; ++q)
          if (q < DB) dx[q] = mfma(wrow[32 * q + n], du, dx[q]);
        if (s.DIN > s.D) {
          df0 = fmaf(wrow[s.D], du, df0);
          df1 = fmaf(wrow[s.D + 1], du, df1);
        }
      }
    }
    TMARK(3);
    // ---- r = dx + ds: history-row grads (LDS atomics per item) and the target-row grad
  #pragma unroll
    for (int q = 0; q < DBM; ++q) {
      if (q >= DB) continue;
      float vt[16];
      // the lane holds dx[d][pair n] for the C-tile rows d = 32 q + crow(0, r, hh)
      // (LDS atomics for the history-row grads: keeping r live until a per-wave round instead
      // costs registers and measured slower, 0.84 vs 0.77 ms at D = H = 128)
  #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = 32 * q + crow(0, r, hh);
        vt[r] = 0.f;
        if (d < s.D && live && n < nj) {
          const float rv = dx[q][r] + ds;
          atomicAdd(&L[g.o_gh + n * g.HD + d], rv * L[g.o_ts + w * s.D + d]);
          vt[r] = rv * L[g.o_hs + n * g.HD + d];
        }
      }
      const float tt = half_reduce_scatter<16>(vt, lane);
      const int d = 32 * q + crow(0, n >> 1, hh);
      if ((n & 1) == 0 && live && d < s.D) {
        if (d < a.IDIM) unsafeAtomicAdd(&gr.et[tgt * a.IDIM + d], tt);
        else unsafeAtomicAdd(&gr.er[a.treg[c] * a.RDIM + (d - a.IDIM)], tt);
      }
    }
    if (s.DIN > s.D) {   // sigmoid, then dist_layer (Linear(2, 2)), summed over the wave's pairs
      df0 += __shfl_xor(df0, 32);
      df1 += __shfl_xor(df1, 32);
      float qv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (live && n < nj && hh == 0) {
        const float* fs = L + g.o_fs + (w * 32 + n) * 4;
        const float q0 = df0 * fs[0] * (1.f - fs[0]), q1 = df1 * fs[1] * (1.f - fs[1]);
        qv[0] = q0 * fs[2];
        qv[1] = q0 * fs[3];
        qv[2] = q1 * fs[2];
        qv[3] = q1 * fs[3];
        qv[4] = q0;
        qv[5] = q1;
      }
  #pragma unroll
      for (int k = 0; k < 6; ++k) {
        const float t = half_sum(qv[k]);
        if (lane == 0 && live) atomicAdd(&L[g.o_gd + k], t);
      }
    }
    TMARK(4);
    constexpr int OWN = (20 + GWT - 1) / GWT;   // dW1 tiles per wave: <= 4 hidden x 5 input blocks
    floatx16 gw[OWN];
#pragma unroll
    for (int q = 0; q < OWN; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) gw[q][r] = 0.f;
    // ---- dW1 = sum over the workgroup's pairs of du x^T: each wave's 32 pairs of du staged in
    // turn (double-buffered: wave rd + 1 stages while every wave consumes wave rd's), x recomputed
    // from the LDS rows by the consumers; every wave accumulates the output tiles it owns (tiles w,
    // w + GWT, w + 2 GWT). One barrier per round.
    const int ntile = g.HB * g.DBX;
    auto stage_du = [&](int buf) {
      float* dst = L + (buf ? g.o_sx : g.o_su) + n * g.UP;
  #pragma unroll
      for (int hb = 0; hb < HBM; ++hb)
  #pragma unroll
        for (int r = 0; r < 16; ++r)
          if (hb < g.HB) dst[crow(hb, r, hh)] = acc[hb][r];
    };
    if (w == 0) stage_du(0);
    __syncthreads();
    for (int rd = 0; rd < GWT; ++rd) {
      if (rd + 1 < GWT && w == rd + 1) stage_du((rd + 1) & 1);
      const float* su = L + ((rd & 1) ? g.o_sx : g.o_su);
  #pragma unroll
      for (int q = 0; q < OWN; ++q) {
        const int tile = w + q * GWT;
        if (tile >= ntile) continue;
        const int ib = tile / g.DBX, xb = tile % g.DBX;
  #pragma unroll 4
        for (int t = 0; t < 16; ++t) {
          const int p = 2 * t + hh;
          gw[q] = mfma(su[p * g.UP + 32 * ib + n], gm_x(s, g, L, rd, p, 32 * xb + n), gw[q]);
        }
      }
      __syncthreads();
    }
    TMARK(5);
    // ---- the unit's dW1 tiles
  #pragma unroll
    for (int q = 0; q < OWN; ++q) {
      const int tile = w + q * GWT;
      if (tile >= ntile) continue;
      const int ib = tile / g.DBX, xb = tile % g.DBX;
  #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = 32 * ib + crow(0, r, hh), d = 32 * xb + n;
        if (i < s.H && d < s.DIN) unsafeAtomicAdd(&gr.w1[int64_t(i) * s.DIN + d], gw[q][r]);
      }
    }
    TMARK(6);
    // ---- the unit's history-row grads (the last dW1 round's barrier ordered every LDS atomic)
    for (int f = tid; f < nj * s.D; f += GWT * 64) {
      const int jj = f / s.D, d = f % s.D;
      const int64_t j = j0 + jj;
      const float v = L[g.o_gh + jj * g.HD + d];
      if (d < a.IDIM) unsafeAtomicAdd(&gr.eh[a.hist[j] * a.IDIM + d], v);
      else unsafeAtomicAdd(&gr.er[a.hreg[j] * a.RDIM + (d - a.IDIM)], v);
    }
    TMARK(7);
  };
  if constexpr (GM_BWD_PERSIST) {
    for (int64_t un = blockIdx.x; un < units; un += gridDim.x) unit(un);
  } else {
    unit(blockIdx.x);
  }
  // ---- flush (once per workgroup): db1 / dw2, dist_layer
  __syncthreads();
  for (int i = tid; i < s.H; i += GWT * 64) {
    unsafeAtomicAdd(&gr.b1[i], Lb[g.o_gb + i]);
    unsafeAtomicAdd(&gr.w2[i], Lb[g.o_gw + i]);
  }
  if (s.DIN > s.D && tid < 6) unsafeAtomicAdd(tid < 4 ? &gr.dw[tid] : &gr.db[tid - 4], Lb[g.o_gd + tid]);
  TMARK(8);
  TFLUSH();
}

// ---------------------------------------------------------------------------------------------
// Generic-shape training kernels (nais_gx.h): embed_dim in (128, 256] or hidden above 128 -- the
// shapes the general kernels above cannot hold (their whole W1 in LDS, hidden <= 128 in
// accumulators). Same math, dropout hash, partials and gradient outputs as gm_forward_kernel /
// gm_backward_kernel; one W1 hidden block at a time in LDS. A unit is (4 * tpw rows, one 32-item
// slice of the shared history); wave w takes rows w * tpw .. w * tpw + tpw - 1, two at a time in
// the forward MFMAs.
//   forward:  per (slice, row) S = sum e, N = sum e (h . t)  (gm_forward_kernel's Sp / Np)
//   backward: pass 1 recomputes the logits (every hidden block) -> e, ds, da per pair; pass 2 per
//             hidden block: z again -> du (ReLU / dropout backward), db1 / dw2 (reduce-scatter
//             into LDS), du^T staged in the wave's LDS rows, dx = W1_blk^T du per 32-dim block
//             consumed at once into the history-row grads (LDS atomics per item) and the target
//             rows (wave-owned LDS rows), the distance features' grads (dims D, D + 1 of dx),
//             and the dW1 tiles (A = du^T, B = x, over the row's 32 pairs) in registers across
//             the wave's rows, added to the gradient once per (wave, hidden block).
// ---------------------------------------------------------------------------------------------
constexpr int GXT_MAX_TPW = 8;
constexpr int GXT_MAX_DBX = (gx::GX_MAX_D + 2 + 31) / 32;   // dW1 column tiles (din <= 258)

struct GxTL {
  int o_w, o_bw, o_h, o_t, o_f, o_l, o_id, o_gh, o_gt, o_du, o_db, o_dw, o_df, o_gd, o_da, fwd, bwd;
  __host__ __device__ GxTL(const gx::Shape& s, int rt) {
    auto al = [](int x) { return (x + 3) & ~3; };
    o_w = 0;
    o_bw = al(32 * s.Q);
    o_h = o_bw + 64;
    o_t = al(o_h + 32 * s.HP);
    o_f = al(o_t + rt * s.D);       // [rt][32][2] distance features f0, f1 of the row's pairs
    o_l = o_f + rt * 64;            // [rt][32][2] their scaled inputs (100 |dlat|, 100 |dlng|)
    o_id = o_l + rt * 64;           // [32] int64 item ids
    fwd = o_id + 64;
    o_gh = fwd;                     // [32][HP] history-row grads of the slice
    o_gt = al(o_gh + 32 * s.HP);    // [rt][D]  target-row grads
    o_du = al(o_gt + rt * s.D);     // [rt][32 pairs][33] du^T of the current hidden block
    o_db = o_du + rt * 32 * 33;     // [HB * 32] db1
    o_dw = o_db + s.HB * 32;        // [HB * 32] dw2
    o_df = o_dw + s.HB * 32;        // [rt][32][2] d(feature) of the row's pairs
    o_gd = o_df + rt * 64;          // [8] dist_layer weight / bias grads
    o_da = o_gd + 8;                // [rt][32][2] ds, da of the row's pairs (pass 1 -> pass 2)
    bwd = o_da + rt * 64;
  }
};

// the unit's operands: the slice's full history rows and ids, the rows' full target rows and the
// pairs' distance features
__device__ __forceinline__ void gxt_stage(const GArgs& a, const gx::Shape& s, const GxTL& o, float* L,
                                          int tid, int64_t c0, int rt, int64_t j0, int nj) {
  for (int f = tid; f < 32 * s.D; f += gx::GX_NT) {
    const int jj = f / s.D, d = f % s.D;
    L[o.o_h + jj * s.HP + d] = jj < nj ? hfull(a, j0 + jj, d) : 0.f;
  }
  if (tid < 32) reinterpret_cast<int64_t*>(L + o.o_id)[tid] = tid < nj ? a.hist[j0 + tid] : -1;
  for (int f = tid; f < rt * s.D; f += gx::GX_NT) {
    const int rq = f / s.D, d = f % s.D;
    const int64_t c = c0 + rq;
    L[o.o_t + f] = c < a.b ? tfull(a, c, d) : 0.f;
  }
  if (s.DIN > s.D) {
    for (int f = tid; f < rt * 32; f += gx::GX_NT) {
      const int rq = f >> 5, jj = f & 31;
      const int64_t c = c0 + rq;
      float f0 = 0.f, f1 = 0.f, l0 = 0.f, l1 = 0.f;
      if (c < a.b && jj < nj) {
        const float* ll = a.ll + c * a.ll_ld + 2 * (j0 + jj);
        l0 = ll[0] * a.dscale;
        l1 = ll[1] * a.dscale;
        // sigmoid(dist_layer(100 ll)), model.py:265, in the scorer's operation order
        f0 = 1.0f / (1.0f + expf(-(l0 * a.dw[0] + l1 * a.dw[1] + a.db[0])));
        f1 = 1.0f / (1.0f + expf(-(l0 * a.dw[2] + l1 * a.dw[3] + a.db[1])));
      }
      L[o.o_f + 2 * f] = f0;
      L[o.o_f + 2 * f + 1] = f1;
      L[o.o_l + 2 * f] = l0;
      L[o.o_l + 2 * f + 1] = l1;
    }
  }
}

struct GxDrop {
  Drop d;
  __device__ __forceinline__ float operator()(uint32_t k, int i) const { return d.factor(k, i); }
};

// pass 1 of both kernels: the attention logit and h . t of the wave's rows' 32 pairs
template <bool DIST, bool DROP>
__device__ __forceinline__ void gxt_logits(const GArgs& a, const gx::Shape& s, const GxTL& o, float* L,
                                           int tid, int lane, int w, int tpw, int64_t c0, int64_t j0,
                                           float (&pa)[GXT_MAX_TPW], float (&sd)[GXT_MAX_TPW]) {
  const int n = lane & 31;
  const GxDrop drop{a.drop};
#pragma unroll
  for (int t = 0; t < GXT_MAX_TPW; ++t) pa[t] = sd[t] = 0.f;
  for (int hb = 0; hb < s.HB; ++hb) {
    __syncthreads();
    gx::stage_w1_block(a.w1, a.b1, a.w2, s, hb, L + o.o_w, L + o.o_bw, tid, gx::GX_NT);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < GXT_MAX_TPW / 2; ++q) {
      if (2 * q >= tpw) continue;
      const int ra = w * tpw + 2 * q;
      const uint32_t ka = DROP ? a.drop.key(uint32_t((c0 + ra) * a.n + j0 + n)) : 0u;
      const uint32_t kb = DROP ? a.drop.key(uint32_t((c0 + ra + 1) * a.n + j0 + n)) : 0u;
      gx::block_logits<true, DIST, DROP>(s, L + o.o_w, L + o.o_bw, L + o.o_h, L + o.o_t + ra * s.D,
                                         L + o.o_t + (ra + 1) * s.D, L + o.o_f + ra * 64,
                                         L + o.o_f + (ra + 1) * 64, lane, hb, hb == 0, pa[2 * q],
                                         pa[2 * q + 1], sd[2 * q], sd[2 * q + 1], drop, ka, kb);
    }
  }
#pragma unroll
  for (int t = 0; t < GXT_MAX_TPW; ++t) {
    pa[t] += __shfl_xor(pa[t], 32);
    sd[t] += __shfl_xor(sd[t], 32);
  }
}

template <bool DIST>
__global__ void __launch_bounds__(gx::GX_NT, 1)
gxt_forward_kernel(GArgs a, float* __restrict__ Sp, float* __restrict__ Np, int tpw) {
  extern __shared__ float4 glds4[];
  float* L = reinterpret_cast<float*>(glds4);
  const gx::Shape s(a.D, a.DIN, a.H);
  const int rt = 4 * tpw;
  const GxTL o(s, rt);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 31;
  const int64_t nrt = (a.b + rt - 1) / rt;
  const int64_t sl = blockIdx.x / nrt, c0 = (blockIdx.x % nrt) * rt, j0 = sl * 32;
  const int nj = (int)(a.n - j0 < 32 ? a.n - j0 : 32);
  gxt_stage(a, s, o, L, tid, c0, rt, j0, nj);
  float pa[GXT_MAX_TPW], sd[GXT_MAX_TPW];
  if (a.drop.on) gxt_logits<DIST, true>(a, s, o, L, tid, lane, w, tpw, c0, j0, pa, sd);
  else gxt_logits<DIST, false>(a, s, o, L, tid, lane, w, tpw, c0, j0, pa, sd);
  const int64_t item = reinterpret_cast<const int64_t*>(L + o.o_id)[n];
#pragma unroll
  for (int t = 0; t < GXT_MAX_TPW; ++t) {
    const int64_t c = c0 + w * tpw + t;
    if (t >= tpw || c >= a.b) continue;
    const float e = n < nj ? expf(pa[t]) * (item != a.target[c] ? 1.f : 0.f) : 0.f;   // model.py:74-78
    const float S = half_sum(e), N = half_sum(e * sd[t]);
    if (lane == 0) {
      Sp[sl * a.b + c] = S;
      Np[sl * a.b + c] = N;
    }
  }
}

template <bool DIST>
__global__ void __launch_bounds__(gx::GX_NT, 1)
gxt_backward_kernel(GArgs a, const float* __restrict__ saved, const float* __restrict__ pred,
                    const float* __restrict__ gpred, GGrads gr, const int32_t* __restrict__ bad_rows,
                    int tpw) {
  if (bad_rows && *bad_rows) return;   // fused step on a NaN batch: no update (see train_loss)
  extern __shared__ float4 glds4[];
  float* L = reinterpret_cast<float*>(glds4);
  const gx::Shape s(a.D, a.DIN, a.H);
  const int rt = 4 * tpw;
  const GxTL o(s, rt);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 31, hh = lane >> 5;
  const int64_t nrt = (a.b + rt - 1) / rt;
  const int64_t sl = blockIdx.x / nrt, c0 = (blockIdx.x % nrt) * rt, j0 = sl * 32;
  const int nj = (int)(a.n - j0 < 32 ? a.n - j0 : 32);
  gxt_stage(a, s, o, L, tid, c0, rt, j0, nj);
  for (int f = tid; f < o.bwd - o.o_gh; f += gx::GX_NT) L[o.o_gh + f] = 0.f;
  // ---- pass 1: logits -> e, ds, da per pair (gm_backward_kernel's formulas)
  float pa[GXT_MAX_TPW], sd[GXT_MAX_TPW];
  if (a.drop.on) gxt_logits<DIST, true>(a, s, o, L, tid, lane, w, tpw, c0, j0, pa, sd);
  else gxt_logits<DIST, false>(a, s, o, L, tid, lane, w, tpw, c0, j0, pa, sd);
  const int64_t item = reinterpret_cast<const int64_t*>(L + o.o_id)[n];
#pragma unroll
  for (int t = 0; t < GXT_MAX_TPW; ++t) {
    float ds = 0.f, da = 0.f;
    const int64_t c = c0 + w * tpw + t;
    if (t < tpw && c < a.b) {
      const float e = n < nj ? expf(pa[t]) * (item != a.target[c] ? 1.f : 0.f) : 0.f;
      const float S = saved[c], N = saved[a.b + c], pc = pred[c];
      const float gl = gpred[c] * pc * (1.f - pc);                // dL/dlogit (sigmoid)
      const float Sb = (a.beta == 0.5f) ? sqrtf(S) : powf(S, a.beta);
      ds = gl / Sb * e;                                             // dlogit / ds_cj
      da = ds * (sd[t] - a.beta * N / S);                           // dlogit / da_cj
    }
    if (t < tpw && lane < 32) {   // both lane halves hold the pair's values
      L[o.o_da + (w * tpw + t) * 64 + 2 * n] = ds;
      L[o.o_da + (w * tpw + t) * 64 + 2 * n + 1] = da;
    }
  }
  // ---- pass 2, per hidden block. Phase A per row: z again -> du (kept in the wave's LDS rows as
  // du^T), db1 / dw2, dx per 32-dim block consumed into the history / target-row grads and the
  // distance features' grads. Phase B per 32-column block of W1: the dW1 tile over every row of
  // the wave (A = du^T, B = x), added to the gradient once per (wave, hidden block, column block).
  const float kscale = a.drop.on ? a.drop.scale : 1.f;
  const int DB = (s.D + 31) / 32, DBX = (s.DIN + 31) / 32;
  for (int hb = 0; hb < s.HB; ++hb) {
    __syncthreads();
    gx::stage_w1_block(a.w1, a.b1, a.w2, s, hb, L + o.o_w, L + o.o_bw, tid, gx::GX_NT);
    __syncthreads();
    const float* Lw = L + o.o_w;
    const float* Lbw = L + o.o_bw;
#pragma unroll 1
    for (int t = 0; t < tpw; ++t) {
      const int rq = w * tpw + t;
      const int64_t c = c0 + rq;
      float* Ldu = L + o.o_du + rq * 32 * 33;
      if (c >= a.b) {   // a row past the batch: du = 0 for phase B
        for (int f = lane; f < 32 * 33; f += 64) Ldu[f] = 0.f;
        continue;
      }
      const float dsp = L[o.o_da + rq * 64 + 2 * n], dap = L[o.o_da + rq * 64 + 2 * n + 1];
      const float* trow = L + o.o_t + rq * s.D;
      floatx16 z = gx::block_z<DIST>(s, Lw, Lbw, L + o.o_h, trow, L + o.o_f + rq * 64, lane);
      const uint32_t key = a.drop.on ? a.drop.key(uint32_t(c * a.n + j0 + n)) : 0u;
      float vb[16], vz[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = gx::crow(0, r, hh);
        float v = z[r];
        if (a.drop.on) v *= a.drop.factor(key, 32 * hb + i);
        // ReLU + dropout backward: v > 0 only where the unit was kept (gm_backward_kernel)
        const float du = v > 0.f ? dap * Lbw[32 + i] * kscale : 0.f;
        z[r] = du;
        vb[r] = du;
        vz[r] = dap * nais_relu(v);
        Ldu[n * 33 + i] = du;                                       // du^T: [pair][hidden]
      }
      const float tb = half_reduce_scatter<16>(vb, lane);
      const float tz = half_reduce_scatter<16>(vz, lane);
      if ((n & 1) == 0) {
        const int i = gx::crow(0, n >> 1, hh);
        atomicAdd(&L[o.o_db + 32 * hb + i], tb);
        atomicAdd(&L[o.o_dw + 32 * hb + i], tz);
      }
      const bool live = n < nj;
#pragma unroll 1
      for (int q = 0; q < DBX; ++q) {
        // dx rows 32 q .. 32 q + 31 (dims; past D: the distance features' d(feature))
        floatx16 dx;
#pragma unroll
        for (int r = 0; r < 16; ++r) dx[r] = 0.f;
        const int col = (32 * q + n) < s.Q ? 32 * q + n : 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) dx = gx::mfma(Lw[gx::crow(0, r, hh) * s.Q + col], z[r], dx);
        float vt[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = 32 * q + gx::crow(0, r, hh);
          vt[r] = 0.f;
          if (d < s.D && live) {
            const float rv = dx[r] + (hb == 0 ? dsp : 0.f);
            atomicAdd(&L[o.o_gh + n * s.HP + d], rv * trow[d]);
            vt[r] = rv * L[o.o_h + n * s.HP + d];
          } else if (DIST && d >= s.D && d < s.DIN && live) {
            L[o.o_df + rq * 64 + 2 * n + (d - s.D)] += dx[r];       // wave-owned row, one lane
          }
        }
        if (q < DB) {
          const float tt = half_reduce_scatter<16>(vt, lane);
          const int d = 32 * q + gx::crow(0, n >> 1, hh);
          if ((n & 1) == 0 && d < s.D) L[o.o_gt + rq * s.D + d] += tt;   // wave-owned row
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // phase B: the wave's dW1 tiles of this hidden block
#pragma unroll 1
    for (int q = 0; q < DBX; ++q) {
      floatx16 gw;
#pragma unroll
      for (int r = 0; r < 16; ++r) gw[r] = 0.f;
      const int k = 32 * q + n;
#pragma unroll 1
      for (int t = 0; t < tpw; ++t) {
        const int rq = w * tpw + t;
        const float* Ldu = L + o.o_du + rq * 32 * 33;
        const float tk = k < s.D ? L[o.o_t + rq * s.D + k] : 0.f;
#pragma unroll 4
        for (int t2 = 0; t2 < 16; ++t2) {
          const int p = 2 * t2 + hh;
          float x = 0.f;
          if (k < s.D) x = L[o.o_h + p * s.HP + k] * tk;
          else if (DIST && k < s.DIN) x = L[o.o_f + rq * 64 + 2 * p + (k - s.D)];
          gw = gx::mfma(Ldu[p * 33 + n], x, gw);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = 32 * hb + gx::crow(0, r, hh);
        if (i < s.H && k < s.DIN) unsafeAtomicAdd(&gr.w1[int64_t(i) * s.DIN + k], gw[r]);
      }
    }
  }
  __syncthreads();
  // ---- the unit's flush: history rows, target rows, db1 / dw2, dist_layer
  for (int f = tid; f < nj * s.D; f += gx::GX_NT) {
    const int jj = f / s.D, d = f % s.D;
    const int64_t j = j0 + jj;
    const float v = L[o.o_gh + jj * s.HP + d];
    if (d < a.IDIM) unsafeAtomicAdd(&gr.eh[a.hist[j] * a.IDIM + d], v);
    else unsafeAtomicAdd(&gr.er[a.hreg[j] * a.RDIM + (d - a.IDIM)], v);
  }
  for (int f = tid; f < rt * s.D; f += gx::GX_NT) {
    const int rq = f / s.D, d = f % s.D;
    const int64_t c = c0 + rq;
    if (c >= a.b) continue;
    const float v = L[o.o_gt + f];
    if (d < a.IDIM) unsafeAtomicAdd(&gr.et[a.target[c] * a.IDIM + d], v);
    else unsafeAtomicAdd(&gr.er[a.treg[c] * a.RDIM + (d - a.IDIM)], v);
  }
  for (int i = tid; i < s.H; i += gx::GX_NT) {
    unsafeAtomicAdd(&gr.b1[i], L[o.o_db + i]);
    unsafeAtomicAdd(&gr.w2[i], L[o.o_dw + i]);
  }
  if (DIST) {   // sigmoid, then dist_layer (Linear(2, 2)), summed over the unit's pairs
    float qv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int f = tid; f < rt * 32; f += gx::GX_NT) {
      const int rq = f >> 5, jj = f & 31;
      if (c0 + rq >= a.b || jj >= nj) continue;
      const float f0 = L[o.o_f + 2 * f], f1 = L[o.o_f + 2 * f + 1];
      const float q0 = L[o.o_df + 2 * f] * f0 * (1.f - f0), q1 = L[o.o_df + 2 * f + 1] * f1 * (1.f - f1);
      const float l0 = L[o.o_l + 2 * f], l1 = L[o.o_l + 2 * f + 1];
      qv[0] += q0 * l0;
      qv[1] += q0 * l1;
      qv[2] += q1 * l0;
      qv[3] += q1 * l1;
      qv[4] += q0;
      qv[5] += q1;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      float v = qv[k];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) atomicAdd(&L[o.o_gd + k], v);
    }
    __syncthreads();
    if (tid < 6) unsafeAtomicAdd(tid < 4 ? &gr.dw[tid] : &gr.db[tid - 4], L[o.o_gd + tid]);
  }
}

size_t g_lds_bytes(const GArgs& a, bool backward, int gw = GW) {
  const GL g(a.D, a.H, a.DIN, gw);
  return size_t(backward ? g.bwd : g.fwd) * sizeof(float);
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
struct TShape {
  int DH, HB;
};

int tvalidate(const nais_params_t* p, TShape* sh) {
  if (!p) return nais_internal_fail(NAIS_E_INVALID, "params is NULL");
  if (p->variant != NAIS_VARIANT_BASIC)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "training step: only NAIS_basic is supported");
  if (!p->embed_history || !p->embed_target || !p->w1 || !p->b1 || !p->w2)
    return nais_internal_fail(NAIS_E_INVALID, "missing parameter pointer");
  const int D = p->embed_dim;
  if (p->item_dim != D || p->din != D)
    return nais_internal_fail(NAIS_E_INVALID, "basic: item_dim == din == embed_dim");
  if (D != 8 && D != 16 && D != 32 && D != 64)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "training step: embed_dim must be 8, 16, 32 or 64");
  if (p->hidden <= 0 || p->hidden > 64)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "training step: hidden must be in [1, 64]");
  sh->DH = D / 2;
  sh->HB = p->hidden > 32 ? 2 : 1;
  return NAIS_OK;
}

TrainArgs targs(const nais_params_t* p, const int64_t* hist, int64_t n, const int64_t* target,
                int64_t b, int js, float dropout_p, uint64_t seed) {
  TrainArgs a;
  a.eh = p->embed_history;
  a.et = p->embed_target;
  a.w1 = p->w1;
  a.b1 = p->b1;
  a.w2 = p->w2;
  a.hist = hist;
  a.target = target;
  a.b = b;
  a.n = n;
  a.H = p->hidden;
  a.D = p->embed_dim;
  a.beta = p->beta;
  a.js = js;
  a.drop = make_drop(dropout_p, seed);
  return a;
}

// Items per slice: about `per_cu` workgroups per CU over the 256 CUs, at most MAX_JS.
int slice_items(int64_t b, int64_t n, int per_cu) {
  const int64_t rb = (b + TROWS - 1) / TROWS;
  const int64_t want = 256 * per_cu;
  int64_t js = (n * rb + want - 1) / want;
  return (int)std::max<int64_t>(1, std::min<int64_t>(MAX_JS, js));
}
constexpr int FWD_PER_CU = 1, BWD_PER_CU = 1;

template <typename K>
void set_lds(K kern, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <int DH, int HB>
int launch_train_forward(const TrainArgs& a, float* Sp, float* Np, hipStream_t st) {
  const size_t lds = size_t(TL<DH, HB>::FWD) * 4;
  auto kern = train_forward_kernel<DH, HB>;
  static bool once = (set_lds(kern, lds), true);
  (void)once;
  dim3 grid((unsigned)((a.b + TROWS - 1) / TROWS), (unsigned)((a.n + a.js - 1) / a.js));
  hipLaunchKernelGGL(kern, grid, dim3(TTHREADS), lds, st, a, Sp, Np);
  return nais_internal_check_launch("train_forward_kernel");
}

template <int DH, int HB>
int launch_train_backward(const TrainArgs& a, const float* saved, const float* pred,
                          const float* gpred, float* Wt, float* Ww, float* Wh, hipStream_t st) {
  const size_t lds = size_t(TL<DH, HB>::BWD) * 4;
  auto kern = train_backward_kernel<DH, HB>;
  static bool once = (set_lds(kern, lds), true);
  (void)once;
  dim3 grid((unsigned)((a.b + TROWS - 1) / TROWS), (unsigned)((a.n + a.js - 1) / a.js));
  hipLaunchKernelGGL(kern, grid, dim3(TTHREADS), lds, st, a, saved, pred, gpred, Wt, Ww, Wh);
  return nais_internal_check_launch("train_backward_kernel");
}

#define NAIS_TRAIN_DISPATCH(FN, SH, ...)                        \
  switch ((SH).DH * 4 + (SH).HB) {                              \
    case 4 * 4 + 1: rc = FN<4, 1>(__VA_ARGS__); break;          \
    case 4 * 4 + 2: rc = FN<4, 2>(__VA_ARGS__); break;          \
    case 8 * 4 + 1: rc = FN<8, 1>(__VA_ARGS__); break;          \
    case 8 * 4 + 2: rc = FN<8, 2>(__VA_ARGS__); break;          \
    case 16 * 4 + 1: rc = FN<16, 1>(__VA_ARGS__); break;        \
    case 16 * 4 + 2: rc = FN<16, 2>(__VA_ARGS__); break;        \
    case 32 * 4 + 1: rc = FN<32, 1>(__VA_ARGS__); break;        \
    default: rc = FN<32, 2>(__VA_ARGS__); break;                \
  }

int check_batch(const int64_t* hist, int64_t n, const int64_t* target, int64_t b) {
  if (b < 0 || n < 0) return nais_internal_fail(NAIS_E_INVALID, "negative b or n");
  if (b > 0 && !target) return nais_internal_fail(NAIS_E_INVALID, "missing target");
  if (n > 0 && !hist) return nais_internal_fail(NAIS_E_INVALID, "missing history");
  if ((b + TROWS - 1) / TROWS > 0x7fffffff) return nais_internal_fail(NAIS_E_UNSUPPORTED, "b too large");
  return NAIS_OK;
}

int hip_rc(hipError_t e, const char* what) {
  if (e == hipSuccess) return NAIS_OK;
  return nais_internal_fail(NAIS_E_HIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
}

// the fused MFMA kernels cover NAIS_basic at D in {8, 16, 32, 64}, H <= 64
// the generic-shape training kernels' shapes (no u cache there: the backward recomputes z)
bool gx_shape(const nais_params_t* p) { return p->embed_dim > G_MAX_D || p->hidden > G_MAX_H; }

bool fast_ok(const nais_params_t* p) {
  const int D = p->embed_dim;
  return p->variant == NAIS_VARIANT_BASIC && (D == 8 || D == 16 || D == 32 || D == 64) &&
         p->item_dim == D && p->din == D && p->hidden >= 1 && p->hidden <= 64;
}

int gvalidate(const nais_params_t* p, const nais_train_side_t* side, int64_t b, int64_t n) {
  if (!p) return nais_internal_fail(NAIS_E_INVALID, "params is NULL");
  if (!p->embed_history || !p->embed_target || !p->w1 || !p->b1 || !p->w2)
    return nais_internal_fail(NAIS_E_INVALID, "missing parameter pointer");
  const int D = p->embed_dim;
  // up to 128 the general kernels, above (embed_dim <= 256, any hidden) the generic-shape ones
  if (D <= 0 || D > gx::GX_MAX_D || p->hidden <= 0)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "training: embed_dim must be in [1, 256], hidden >= 1");
  switch (p->variant) {
    case NAIS_VARIANT_BASIC:
      if (p->item_dim != D || p->din != D)
        return nais_internal_fail(NAIS_E_INVALID, "basic: item_dim == din == embed_dim");
      break;
    case NAIS_VARIANT_REGION:
    case NAIS_VARIANT_REGION_DISTANCE: {
      if (p->item_dim + p->region_dim != D || p->item_dim <= 0 || !p->embed_region)
        return nais_internal_fail(NAIS_E_INVALID, "region: item_dim + region_dim == embed_dim, embed_region set");
      const int want = p->variant == NAIS_VARIANT_REGION ? D : D + 2;
      if (p->din != want) return nais_internal_fail(NAIS_E_INVALID, "region: din must be embed_dim (+2 with distance)");
      if (p->variant == NAIS_VARIANT_REGION_DISTANCE && (!p->dist_w || !p->dist_b))
        return nais_internal_fail(NAIS_E_INVALID, "region_distance: dist_w / dist_b missing");
      if (b > 0 && n > 0 && (!side || !side->hist_region || !side->target_region))
        return nais_internal_fail(NAIS_E_INVALID, "region variants need side->hist_region / target_region");
      if (p->variant == NAIS_VARIANT_REGION_DISTANCE && b > 0 && n > 0 &&
          (!side->target_lat_long || side->latlon_ld < 2 * n))
        return nais_internal_fail(NAIS_E_INVALID, "region_distance needs side->target_lat_long [b, n, 2]");
      break;
    }
    case NAIS_VARIANT_DISTANCE:
      if (p->item_dim != D || p->din != D + 2 || !p->dist_w || !p->dist_b)
        return nais_internal_fail(NAIS_E_INVALID, "distance: item_dim == embed_dim, din == embed_dim + 2, dist_layer set");
      if (b > 0 && n > 0 && (!side || !side->target_lat_long || side->latlon_ld < 2 * n))
        return nais_internal_fail(NAIS_E_INVALID, "distance needs side->target_lat_long [b, n, 2]");
      break;
    default:
      return nais_internal_fail(NAIS_E_UNSUPPORTED, "training: unknown variant");
  }
  return NAIS_OK;
}

int g_slice_items(int64_t, int64_t) { return 32; }   // one 32-pair MFMA tile per wave and slice

GArgs gargs(const nais_params_t* p, const nais_train_side_t* side, const int64_t* hist, int64_t n,
            const int64_t* target, int64_t b, float dropout_p, uint64_t seed) {
  GArgs a;
  a.eh = p->embed_history;
  a.et = p->embed_target;
  a.er = p->embed_region;
  a.w1 = p->w1;
  a.b1 = p->b1;
  a.w2 = p->w2;
  a.dw = p->dist_w;
  a.db = p->dist_b;
  a.hist = hist;
  a.target = target;
  a.hreg = side ? side->hist_region : nullptr;
  a.treg = side ? side->target_region : nullptr;
  a.ll = side ? side->target_lat_long : nullptr;
  a.ll_ld = side ? side->latlon_ld : 0;
  a.b = b;
  a.n = n;
  a.D = p->embed_dim;
  const bool reg = p->variant == NAIS_VARIANT_REGION || p->variant == NAIS_VARIANT_REGION_DISTANCE;
  a.IDIM = reg ? p->item_dim : p->embed_dim;
  a.RDIM = reg ? p->region_dim : 0;
  a.H = p->hidden;
  a.DIN = p->din;
  a.variant = p->variant;
  a.beta = p->beta;
  a.dscale = p->variant == NAIS_VARIANT_DISTANCE ? 1000.f : 100.f;   // model.py:369 / :265
  a.js = g_slice_items(b, n);
  a.drop = make_drop(dropout_p, seed);
  a.ucache = nullptr;
  return a;
}

size_t g_workspace(int64_t b, int64_t n) {
  if (b <= 0 || n <= 0) return 0;
  const int64_t ns = (n + g_slice_items(b, n) - 1) / g_slice_items(b, n);
  return size_t(2 * ns * b) * sizeof(float);
}

int device_cus() {
  static int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return cus;
  }();
  return n;
}

// The compile-time instantiations of the general kernels: (D, H, extra input dims). Other shapes
// run the runtime-shaped <HBM> kernels.
#define NAIS_GM_SHAPES(X) X(4, 128, 128, 0) X(4, 128, 128, 2) X(2, 64, 64, 0) X(2, 64, 64, 2)
// the backward at D = 128 with the 2 distance inputs spills (256 VGPRs + 36): runtime-shaped there
#define NAIS_GM_SHAPES_BWD(X) X(4, 128, 128, 0) X(2, 64, 64, 0) X(2, 64, 64, 2)

// rows per wave of the generic training kernels: the most of 8 / 4 / 2 whose LDS image fits
int gxt_tpw(const GArgs& a, bool backward) {
  const gx::Shape s(a.D, a.DIN, a.H);
  for (int tpw = GXT_MAX_TPW; tpw >= 2; tpw /= 2) {
    const GxTL o(s, 4 * tpw);
    if (size_t(backward ? o.bwd : o.fwd) * 4 <= 160 * 1024) return tpw;
  }
  return 0;
}

bool gxt_big(const GArgs& a) { return a.D > G_MAX_D || a.H > G_MAX_H; }

int gxt_forward(const GArgs& a, float* Sp, float* Np, hipStream_t st) {
  const int tpw = gxt_tpw(a, false);
  if (!tpw) return nais_internal_fail(NAIS_E_UNSUPPORTED, "training: shape exceeds the generic kernels' LDS budget");
  const gx::Shape s(a.D, a.DIN, a.H);
  const size_t lds = size_t(GxTL(s, 4 * tpw).fwd) * 4;
  static bool once = (set_lds(gxt_forward_kernel<false>, 160 * 1024), set_lds(gxt_forward_kernel<true>, 160 * 1024), true);
  (void)once;
  const int64_t units = ((a.b + 4 * tpw - 1) / (4 * tpw)) * ((a.n + 31) / 32);
  if (a.DIN > a.D)
    hipLaunchKernelGGL(gxt_forward_kernel<true>, dim3((unsigned)units), dim3(gx::GX_NT), lds, st, a, Sp, Np, tpw);
  else
    hipLaunchKernelGGL(gxt_forward_kernel<false>, dim3((unsigned)units), dim3(gx::GX_NT), lds, st, a, Sp, Np, tpw);
  return nais_internal_check_launch("gxt_forward_kernel");
}

int gxt_backward(const GArgs& a, const float* saved, const float* pred, const float* gpred,
                 const GGrads& g, hipStream_t st, const int32_t* bad_rows) {
  const int tpw = gxt_tpw(a, true);
  if (!tpw) return nais_internal_fail(NAIS_E_UNSUPPORTED, "training: shape exceeds the generic kernels' LDS budget");
  const gx::Shape s(a.D, a.DIN, a.H);
  const size_t lds = size_t(GxTL(s, 4 * tpw).bwd) * 4;
  static bool once = (set_lds(gxt_backward_kernel<false>, 160 * 1024), set_lds(gxt_backward_kernel<true>, 160 * 1024), true);
  (void)once;
  const int64_t units = ((a.b + 4 * tpw - 1) / (4 * tpw)) * ((a.n + 31) / 32);
  if (a.DIN > a.D)
    hipLaunchKernelGGL(gxt_backward_kernel<true>, dim3((unsigned)units), dim3(gx::GX_NT), lds, st, a, saved, pred,
                       gpred, g, bad_rows, tpw);
  else
    hipLaunchKernelGGL(gxt_backward_kernel<false>, dim3((unsigned)units), dim3(gx::GX_NT), lds, st, a, saved, pred,
                       gpred, g, bad_rows, tpw);
  return nais_internal_check_launch("gxt_backward_kernel");
}

template <int GWT>
int g_forward_launch(const GArgs& a, float* Sp, float* Np, hipStream_t st, int64_t units, int sl0,
                     int trows = 0) {
  const size_t lds = g_lds_bytes(a, false, GWT);
#define NAIS_GM_LDS(HBM, DC, HC, XC) set_lds(gm_forward_kernel<HBM, DC, HC, XC, GWT>, 160 * 1024),
  static bool once = (NAIS_GM_SHAPES(NAIS_GM_LDS) set_lds(gm_forward_kernel<4, 0, 0, 0, GWT>, 160 * 1024),
                      set_lds(gm_forward_kernel<2, 0, 0, 0, GWT>, 160 * 1024), true);
#undef NAIS_GM_LDS
  (void)once;
  // persistent: one workgroup per CU (the LDS image holds one), units strided over the grid
  dim3 grid((unsigned)std::min<int64_t>(units, device_cus()));
#define NAIS_GM_FWD(HBM, DC, HC, XC)                                                        \
  if (a.D == DC && a.H == HC && a.DIN == DC + XC) {                                        \
    hipLaunchKernelGGL((gm_forward_kernel<HBM, DC, HC, XC, GWT>), grid, dim3(GWT * 64), lds, st, a, \
                       Sp, Np, sl0, trows);                                                \
    return nais_internal_check_launch("gm_forward_kernel");                                \
  }
  NAIS_GM_SHAPES(NAIS_GM_FWD)
#undef NAIS_GM_FWD
  if (a.H > 64)
    hipLaunchKernelGGL((gm_forward_kernel<4, 0, 0, 0, GWT>), grid, dim3(GWT * 64), lds, st, a, Sp, Np, sl0,
                       trows);
  else
    hipLaunchKernelGGL((gm_forward_kernel<2, 0, 0, 0, GWT>), grid, dim3(GWT * 64), lds, st, a, Sp, Np, sl0,
                       trows);
  return nais_internal_check_launch("gm_forward_kernel");
}

constexpr int GM_TAIL = 4;   // rows per workgroup of the short-slice launches; 0 = one launch each
// (config-3 step at D = H = 128, interleaved: 4 rows 0.487 / 0.485 ms, 2 rows 0.558 / 0.566, 6 rows
// 0.497 / 0.497, 8 rows 0.498 / 0.497 -- profiles/r5/train_tail)
// The general kernels' units are (row tile, 32-item slice) workgroups, one per CU (LDS). When the
// short last slice (n % 32 items) pushes the unit count into one more round of workgroups over the
// CUs -- config 3: 85 row tiles x 7 slices = 595 units = 2.3 rounds of 256, the third almost empty
// but as long as a full one, since a slice of 12 items costs the MFMAs of 32 -- that slice runs as
// a second launch of GM_TAIL-row workgroups (one wave per SIMD, a third of a unit's waves)
// after the full slices' exactly-filled rounds (the backward; see g_forward). Returns the number of
// full slices to launch first (== the slice count when no split pays).
int64_t g_split_slices(const GArgs& a) {
  const int64_t nrt = (a.b + GW - 1) / GW, nsl = (a.n + 31) / 32, nfull = a.n / 32;
  const int64_t cus = device_cus();
  if (GM_TAIL <= 0 || nfull == 0 || nsl == nfull) return nsl;
  const char* off = getenv("NAIS_GM_TAIL");   // "0": one launch (tests compare both forms)
  if (off && off[0] == '0' && off[1] == 0) return nsl;
  const int64_t rounds_all = (nrt * nsl + cus - 1) / cus, rounds_full = (nrt * nfull + cus - 1) / cus;
  return rounds_full < rounds_all ? nfull : nsl;
}

// The forward stays one persistent launch: its workgroups stage W1 once for all their units, so
// the short slice's units ride on workgroups that already hold it (A/B, config 3 at D = H = 128:
// split 0.129 ms vs 0.110 ms -- a 4-row tail workgroup pays a whole W1 staging for one unit).
// Inside that launch the short slice's units are GM_TAIL-row tiles when the backward splits
// (same criterion, g_split_slices): config 3's 85 twelve-row short units become 255 four-row ones,
// one per workgroup's last round instead of a full-length third round on 85 of them.
// NAIS_GM_FWD_TAIL=0: twelve-row short units (A/B).
int g_forward(const GArgs& a, float* Sp, float* Np, hipStream_t st) {
  if (gxt_big(a)) return gxt_forward(a, Sp, Np, st);
  const int64_t nrt = (a.b + GW - 1) / GW, nsl = (a.n + 31) / 32;
  static const bool fwd_tail = [] {
    const char* e = getenv("NAIS_GM_FWD_TAIL");
    return !(e && e[0] == '0');
  }();
  const int trows = (fwd_tail && GM_TAIL > 0 && g_split_slices(a) < nsl) ? GM_TAIL : 0;
  const int64_t units = trows > 0 ? nrt * (nsl - 1) + (a.b + trows - 1) / trows : nrt * nsl;
  return g_forward_launch<GW>(a, Sp, Np, st, units, 0, trows);
}

template <int GWT>
int g_backward_launch(const GArgs& a, const float* saved, const float* pred, const float* gpred,
                      const GGrads& g, hipStream_t st, const int32_t* bad_rows, int64_t units, int sl0) {
  const size_t lds = g_lds_bytes(a, true, GWT);
#define NAIS_GM_LDS(HBM, DC, HC, XC) set_lds(gm_backward_kernel<HBM, DC, HC, XC, GWT>, 160 * 1024),
  static bool once = (NAIS_GM_SHAPES_BWD(NAIS_GM_LDS) set_lds(gm_backward_kernel<4, 0, 0, 0, GWT>, 160 * 1024),
                      set_lds(gm_backward_kernel<2, 0, 0, 0, GWT>, 160 * 1024), true);
#undef NAIS_GM_LDS
  (void)once;
  dim3 grid((unsigned)(GM_BWD_PERSIST ? std::min<int64_t>(units, device_cus()) : units));
#define NAIS_GM_BWD(HBM, DC, HC, XC)                                                        \
  if (a.D == DC && a.H == HC && a.DIN == DC + XC) {                                        \
    hipLaunchKernelGGL((gm_backward_kernel<HBM, DC, HC, XC, GWT>), grid, dim3(GWT * 64), lds, st, a, \
                       saved, pred, gpred, g, bad_rows, sl0);                              \
    return nais_internal_check_launch("gm_backward_kernel");                               \
  }
  NAIS_GM_SHAPES_BWD(NAIS_GM_BWD)
#undef NAIS_GM_BWD
  if (a.H > 64)
    hipLaunchKernelGGL((gm_backward_kernel<4, 0, 0, 0, GWT>), grid, dim3(GWT * 64), lds, st, a, saved,
                       pred, gpred, g, bad_rows, sl0);
  else
    hipLaunchKernelGGL((gm_backward_kernel<2, 0, 0, 0, GWT>), grid, dim3(GWT * 64), lds, st, a, saved,
                       pred, gpred, g, bad_rows, sl0);
  return nais_internal_check_launch("gm_backward_kernel");
}

int g_backward(const GArgs& a, const float* saved, const float* pred, const float* gpred,
               const GGrads& g, hipStream_t st, const int32_t* bad_rows = nullptr) {
  if (gxt_big(a)) return gxt_backward(a, saved, pred, gpred, g, st, bad_rows);
  const int64_t nrt = (a.b + GW - 1) / GW, nsl = (a.n + 31) / 32;
  const int64_t first = GM_BWD_PERSIST ? nsl : g_split_slices(a);
  int rc = g_backward_launch<GW>(a, saved, pred, gpred, g, st, bad_rows, nrt * first, 0);
  if (rc || first == nsl || GM_TAIL <= 0) return rc;
  constexpr int TW_ = GM_TAIL > 0 ? GM_TAIL : 1;
  return g_backward_launch<TW_>(a, saved, pred, gpred, g, st, bad_rows, (a.b + TW_ - 1) / TW_, (int)first);
}

}  // namespace

extern "C" {

namespace {
// the caller's u cache of the autograd split (nais_train_side_t::ucache), when large enough
float* side_ucache(const nais_params_t* params, const nais_train_side_t* side, int64_t b, int64_t n) {
  if (!side || !side->ucache || fast_ok(params) || gx_shape(params) || b <= 0 || n <= 0) return nullptr;
  const size_t need = ucache_bytes(params->hidden, b, n);
  return (need <= UCACHE_MAX_BYTES && side->ucache_bytes >= need) ? side->ucache : nullptr;
}

// the fused step's u cache (general kernels only), after saved / gpred / pred / the partials
size_t step_ucache_bytes(const nais_params_t* params, int64_t b, int64_t n) {
  if (!params || b <= 0 || n <= 0 || fast_ok(params) || gx_shape(params)) return 0;
  const size_t u = ucache_bytes(params->hidden, b, n);
  return u <= UCACHE_MAX_BYTES ? u : 0;
}
size_t step_ucache_offset(const nais_params_t* params, int64_t b, int64_t n) {
  const size_t o = nais_train_workspace_size(params, b, n) + size_t(4 * b) * sizeof(float);
  return (o + 255) & ~size_t(255);
}
}  // namespace

size_t nais_train_ucache_size(const nais_params_t* params, int64_t b, int64_t n) {
  if (!params || b <= 0 || n <= 0 || fast_ok(params) || gx_shape(params)) return 0;
  const size_t u = ucache_bytes(params->hidden, b, n);
  return u <= UCACHE_MAX_BYTES ? u : 0;
}

size_t nais_train_step_workspace_size(const nais_params_t* params, int64_t b, int64_t n) {
  if (!params || b <= 0) return 0;
  const size_t u = step_ucache_bytes(params, b, n);   // fast or general (+ the general u cache)
  return u ? step_ucache_offset(params, b, n) + u
           : nais_train_workspace_size(params, b, n) + size_t(4 * b) * sizeof(float);
}

namespace {
int32_t train_step_impl(const nais_params_t* params, const nais_train_side_t* side,
                        const nais_adagrad_state_t* opt, const nais_adagrad_side_t* opt_side,
                        const int64_t* hist, int64_t n, const int64_t* target, const float* labels,
                        int64_t b, float dropout_p, uint64_t seed, float* loss_sum,
                        int32_t* bad_rows, float* pred, void* workspace, size_t workspace_bytes,
                        void* stream) {
  TShape sh{0, 0};
  const bool fast = params && fast_ok(params);
  int rc = fast ? tvalidate(params, &sh) : gvalidate(params, side, b, n);
  if (rc) return rc;
  const bool region = params->variant == NAIS_VARIANT_REGION ||
                      params->variant == NAIS_VARIANT_REGION_DISTANCE;
  const bool distv = params->variant == NAIS_VARIANT_REGION_DISTANCE ||
                     params->variant == NAIS_VARIANT_DISTANCE;
  if ((region || distv) &&
      (!opt_side || (region && (!opt_side->sum_embed_region || !opt_side->grad_embed_region)) ||
       (distv && (!opt_side->sum_dist_w || !opt_side->sum_dist_b || !opt_side->grad_dist))))
    return nais_internal_fail(NAIS_E_INVALID, "nais_adagrad_side_t: missing buffer for the variant's "
                                              "embed_region / dist_layer");
  if ((rc = check_batch(hist, n, target, b))) return rc;
  if (!(dropout_p >= 0.f && dropout_p <= 1.f))
    return nais_internal_fail(NAIS_E_INVALID, "dropout_p must be in [0, 1]");
  if (!opt || !loss_sum || !bad_rows || (b > 0 && !labels))
    return nais_internal_fail(NAIS_E_INVALID, "missing opt / loss_sum / bad_rows / labels");
  if (!opt->sum_embed_history || !opt->sum_embed_target || !opt->sum_w1 || !opt->sum_b1 ||
      !opt->sum_w2 || !opt->grad_embed_history || !opt->grad_embed_target || !opt->grad_small ||
      !opt->stamp_embed_history || !opt->stamp_embed_target)
    return nais_internal_fail(NAIS_E_INVALID, "nais_adagrad_state_t: missing buffer");
  if (opt->step < 1) return nais_internal_fail(NAIS_E_INVALID, "opt->step must be >= 1");
  if (b == 0) return NAIS_OK;
  if (!workspace || workspace_bytes < nais_train_step_workspace_size(params, b, n))
    return nais_internal_fail(NAIS_E_WORKSPACE, "workspace too small (nais_train_step_workspace_size)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* ws = static_cast<float*>(workspace);
  float* saved = ws;            // [2b]
  float* gpred = ws + 2 * b;    // [b]
  float* own_pred = ws + 3 * b; // [b]
  float* part = ws + 4 * b;     // forward partials, then backward partials
  if (!pred) pred = own_pred;
  const int D = params->embed_dim, H = params->hidden, DIN = params->din;
  const int RD = region ? params->item_dim : D;   // embed_history / embed_target row width
  int64_t ns = 0, rb = (b + TROWS - 1) / TROWS;
  int js = 1;
  GArgs ga{};
  if (n > 0) {
    if (fast) {
      js = slice_items(b, n, FWD_PER_CU);
    } else {
      ga = gargs(params, side, hist, n, target, b, dropout_p, seed);
      js = ga.js;
      if (step_ucache_bytes(params, b, n))
        ga.ucache = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                             step_ucache_offset(params, b, n));
    }
    ns = (n + js - 1) / js;
    if (ns > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "history too long for the grid");
  }
  const TrainArgs a = targs(params, hist, n, target, b, js, dropout_p, seed);
  // 1. forward partials, 2. loss + dL/dpred
  if (n > 0) {
    if (fast) {
      NAIS_TRAIN_DISPATCH(launch_train_forward, sh, a, part, part + ns * b, st);
    } else {
      rc = g_forward(ga, part, part + ns * b, st);
    }
    if (rc) return rc;
  }
  hipLaunchKernelGGL(train_loss_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, st,
                     part, part + ns * b, (int)ns, b, n, params->beta, labels, pred, saved, gpred,
                     loss_sum, bad_rows);
  if ((rc = nais_internal_check_launch("train_loss_kernel"))) return rc;
  // 3. backward partials, 4. reduce into the zero-maintained gradient scratch
  if (n > 0 && !fast) {   // general kernels add straight into the scratch
    float* gs = opt->grad_small;
    float* gd = distv ? opt_side->grad_dist : nullptr;
    const GGrads g{opt->grad_embed_history, opt->grad_embed_target,
                   region ? opt_side->grad_embed_region : nullptr, gs, gs + int64_t(H) * DIN,
                   gs + int64_t(H) * DIN + H, gd, gd ? gd + 4 : nullptr};
    if ((rc = g_backward(ga, saved, pred, gpred, g, st, bad_rows))) return rc;
  } else if (n > 0) {
    float* Wt = part;
    float* Ww = Wt + ns * b * D;
    float* Wh = Ww + ns * rb * (int64_t(H) * D + 2 * H);
    NAIS_TRAIN_DISPATCH(launch_train_backward, sh, a, saved, pred, gpred, Wt, Ww, Wh, st);
    if (rc) return rc;
    const int64_t total = (int64_t(H) * D + 2 * H) * REDUCE_KS + b * D + n * D;
    float* gs = opt->grad_small;
    hipLaunchKernelGGL(train_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       st, Wt, Ww, Wh, b, n, D, H, (int)ns, (int)rb, hist, target,
                       opt->grad_embed_history, opt->grad_embed_target, gs, gs + int64_t(H) * D,
                       gs + int64_t(H) * D + H, bad_rows);
    if ((rc = nais_internal_check_launch("train_reduce_kernel"))) return rc;
  }
  // 5. Adagrad (run.py:89) straight from the scratch, which it zeroes again
  StepOpt o;
  o.p_eh = const_cast<float*>(params->embed_history);
  o.p_et = const_cast<float*>(params->embed_target);
  o.p_small[0] = const_cast<float*>(params->w1);
  o.p_small[1] = const_cast<float*>(params->b1);
  o.p_small[2] = const_cast<float*>(params->w2);
  o.s_eh = opt->sum_embed_history;
  o.s_et = opt->sum_embed_target;
  o.s_small[0] = opt->sum_w1;
  o.s_small[1] = opt->sum_b1;
  o.s_small[2] = opt->sum_w2;
  o.g_eh = opt->grad_embed_history;
  o.g_et = opt->grad_embed_target;
  o.g_small = opt->grad_small;
  o.st_eh = opt->stamp_embed_history;
  o.st_et = opt->stamp_embed_target;
  o.clr = float(double(opt->lr) / (1.0 + double(opt->step - 1) * double(opt->lr_decay)));
  o.wd = opt->weight_decay;
  o.eps = opt->eps;
  o.tag = int32_t(opt->step);
  const int64_t wsz = int64_t(H) * DIN + 2 * H;
  const int64_t dense = opt->weight_decay != 0.f ? params->num_pois : 0;
  const int64_t rows = dense ? 2 * dense : n + b;
  const int64_t blocks = (wsz + 255) / 256 + (rows + 3) / 4;
  hipLaunchKernelGGL(step_adagrad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, o, H, DIN, RD,
                     hist, n, target, b, dense, bad_rows);
  if ((rc = nais_internal_check_launch("step_adagrad_kernel"))) return rc;
  if (region) {   // every row of embed_region (its batch rows are a few region ids)
    const int64_t ne = int64_t(params->num_regions) * params->region_dim;
    hipLaunchKernelGGL(step_adagrad_dense_kernel, dim3((unsigned)std::min<int64_t>((ne + 255) / 256, 1024)),
                       dim3(256), 0, st, const_cast<float*>(params->embed_region),
                       opt_side->sum_embed_region, opt_side->grad_embed_region, ne, o.clr, o.wd, o.eps,
                       bad_rows);
    if ((rc = nais_internal_check_launch("step_adagrad_dense_kernel"))) return rc;
  }
  if (distv) {    // dist_layer weight [2, 2] and bias [2]
    hipLaunchKernelGGL(step_adagrad_dense_kernel, dim3(1), dim3(64), 0, st,
                       const_cast<float*>(params->dist_w), opt_side->sum_dist_w, opt_side->grad_dist,
                       int64_t(4), o.clr, o.wd, o.eps, bad_rows);
    hipLaunchKernelGGL(step_adagrad_dense_kernel, dim3(1), dim3(64), 0, st,
                       const_cast<float*>(params->dist_b), opt_side->sum_dist_b, opt_side->grad_dist + 4,
                       int64_t(2), o.clr, o.wd, o.eps, bad_rows);
    if ((rc = nais_internal_check_launch("step_adagrad_dense_kernel"))) return rc;
  }
  return NAIS_OK;
}
}  // namespace

int32_t nais_train_step(const nais_params_t* params, const nais_adagrad_state_t* opt,
                        const int64_t* hist, int64_t n, const int64_t* target, const float* labels,
                        int64_t b, float dropout_p, uint64_t seed, float* loss_sum,
                        int32_t* bad_rows, float* pred, void* workspace, size_t workspace_bytes,
                        void* stream) {
  if (params && params->variant != NAIS_VARIANT_BASIC)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "nais_train_step: NAIS_basic only (use nais_train_step_ex)");
  return train_step_impl(params, nullptr, opt, nullptr, hist, n, target, labels, b, dropout_p, seed,
                         loss_sum, bad_rows, pred, workspace, workspace_bytes, stream);
}

int32_t nais_train_step_ex(const nais_params_t* params, const nais_train_side_t* side,
                           const nais_adagrad_state_t* opt, const nais_adagrad_side_t* opt_side,
                           const int64_t* hist, int64_t n, const int64_t* target, const float* labels,
                           int64_t b, float dropout_p, uint64_t seed, float* loss_sum,
                           int32_t* bad_rows, float* pred, void* workspace, size_t workspace_bytes,
                           void* stream) {
  return train_step_impl(params, side, opt, opt_side, hist, n, target, labels, b, dropout_p, seed,
                         loss_sum, bad_rows, pred, workspace, workspace_bytes, stream);
}

int32_t nais_make_train_batch(const int64_t* indptr, const int64_t* indices, int64_t user,
                              int64_t n, int64_t num_pois, int32_t num_ng, uint64_t seed,
                              int64_t* hist, int64_t* target, float* labels, int32_t* err,
                              void* stream) {
  if (!indptr || !indices || user < 0 || n < 0 || num_ng < 0 || num_pois <= 0)
    return nais_internal_fail(NAIS_E_INVALID, "bad arguments");
  if (num_pois > 0x7fffffffll || n > 0x7fffffffll)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "num_pois / n must fit 31 bits");
  if (n * (int64_t(num_ng) + 1) > num_pois)
    return nais_internal_fail(NAIS_E_INVALID, "not enough negatives: n * (1 + num_ng) > num_pois");
  if (n == 0) return NAIS_OK;
  if (!hist || !target || !labels) return nais_internal_fail(NAIS_E_INVALID, "NULL output");
  hipLaunchKernelGGL(make_batch_kernel, dim3(1), dim3(BATCH_THREADS), 0,
                     reinterpret_cast<hipStream_t>(stream), indptr, indices, user, n, num_pois,
                     (int)num_ng, mix32(uint32_t(seed) ^ 0x85ebca6bu),
                     mix32(uint32_t(seed >> 32) ^ uint32_t(seed) * 0x9e3779b9u), hist, target,
                     labels, err);
  return nais_internal_check_launch("make_batch_kernel");
}

size_t nais_train_workspace_size(const nais_params_t* params, int64_t b, int64_t n) {
  if (!params || b <= 0 || n <= 0) return 0;
  if (!fast_ok(params)) return g_workspace(b, n);
  const int js = slice_items(b, n, FWD_PER_CU);
  const int64_t ns = (n + js - 1) / js, rb = (b + TROWS - 1) / TROWS;
  const int64_t D = params->embed_dim, H = params->hidden;
  const int64_t fwd = 2 * ns * b;
  const int64_t bwd = ns * b * D + ns * rb * (H * D + 2 * H) + rb * n * D;
  return size_t(std::max(fwd, bwd)) * sizeof(float);
}

int32_t nais_train_forward_ex(const nais_params_t* params, const nais_train_side_t* side,
                              const int64_t* hist, int64_t n, const int64_t* target, int64_t b,
                              float dropout_p, uint64_t seed, float* pred, float* saved,
                              int32_t* nan_count, void* workspace, size_t workspace_bytes,
                              void* stream) {
  if (params && fast_ok(params))
    return nais_train_forward(params, hist, n, target, b, dropout_p, seed, pred, saved, nan_count,
                              workspace, workspace_bytes, stream);
  int rc = gvalidate(params, side, b, n);
  if (rc) return rc;
  if ((rc = check_batch(hist, n, target, b))) return rc;
  if (!(dropout_p >= 0.f && dropout_p <= 1.f))
    return nais_internal_fail(NAIS_E_INVALID, "dropout_p must be in [0, 1]");
  if (b == 0) return NAIS_OK;
  if (!pred || !saved) return nais_internal_fail(NAIS_E_INVALID, "missing pred/saved");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) {
    hipLaunchKernelGGL(train_finalize_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, st,
                       nullptr, nullptr, 0, b, n, params->beta, pred, saved, nan_count);
    return nais_internal_check_launch("train_finalize_kernel");
  }
  GArgs a = gargs(params, side, hist, n, target, b, dropout_p, seed);
  a.ucache = side_ucache(params, side, b, n);
  const int64_t ns = (n + a.js - 1) / a.js;
  if (ns > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "history too long for the grid");
  if (!workspace || workspace_bytes < g_workspace(b, n))
    return nais_internal_fail(NAIS_E_WORKSPACE, "workspace too small (nais_train_workspace_size)");
  float* Sp = static_cast<float*>(workspace);
  float* Np = Sp + ns * b;
  if ((rc = g_forward(a, Sp, Np, st))) return rc;
  hipLaunchKernelGGL(train_finalize_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, st,
                     Sp, Np, (int)ns, b, n, params->beta, pred, saved, nan_count);
  return nais_internal_check_launch("train_finalize_kernel");
}

int32_t nais_train_backward_ex(const nais_params_t* params, const nais_train_side_t* side,
                               const int64_t* hist, int64_t n, const int64_t* target, int64_t b,
                               float dropout_p, uint64_t seed, const float* pred,
                               const float* saved, const float* grad_pred,
                               const nais_train_grads_t* grads, void* workspace,
                               size_t workspace_bytes, void* stream) {
  if (!grads) return nais_internal_fail(NAIS_E_INVALID, "grads is NULL");
  if (params && fast_ok(params))
    return nais_train_backward(params, hist, n, target, b, dropout_p, seed, pred, saved, grad_pred,
                               grads->embed_history, grads->embed_target, grads->w1, grads->b1,
                               grads->w2, workspace, workspace_bytes, stream);
  int rc = gvalidate(params, side, b, n);
  if (rc) return rc;
  if ((rc = check_batch(hist, n, target, b))) return rc;
  if (!(dropout_p >= 0.f && dropout_p <= 1.f))
    return nais_internal_fail(NAIS_E_INVALID, "dropout_p must be in [0, 1]");
  if (b == 0 || n == 0) return NAIS_OK;
  if (!pred || !saved || !grad_pred || !grads->embed_history || !grads->embed_target || !grads->w1 ||
      !grads->b1 || !grads->w2)
    return nais_internal_fail(NAIS_E_INVALID, "missing pred/saved/grad pointer");
  if ((params->variant == NAIS_VARIANT_REGION || params->variant == NAIS_VARIANT_REGION_DISTANCE) &&
      !grads->embed_region)
    return nais_internal_fail(NAIS_E_INVALID, "region variants need grads->embed_region");
  if (params->variant == NAIS_VARIANT_REGION_DISTANCE && (!grads->dist_w || !grads->dist_b))
    return nais_internal_fail(NAIS_E_INVALID, "region_distance needs grads->dist_w / dist_b");
  if (params->variant == NAIS_VARIANT_DISTANCE && (!grads->dist_w || !grads->dist_b))
    return nais_internal_fail(NAIS_E_INVALID, "distance needs grads->dist_w / dist_b");
  (void)workspace;
  (void)workspace_bytes;
  GArgs a = gargs(params, side, hist, n, target, b, dropout_p, seed);
  a.ucache = side_ucache(params, side, b, n);
  if ((n + a.js - 1) / a.js > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "history too long for the grid");
  const GGrads g{grads->embed_history, grads->embed_target, grads->embed_region, grads->w1,
                 grads->b1, grads->w2, grads->dist_w, grads->dist_b};
  return g_backward(a, saved, pred, grad_pred, g, reinterpret_cast<hipStream_t>(stream));
}

int32_t nais_train_forward(const nais_params_t* params, const int64_t* hist, int64_t n,
                           const int64_t* target, int64_t b, float dropout_p, uint64_t seed,
                           float* pred, float* saved, int32_t* nan_count, void* workspace,
                           size_t workspace_bytes, void* stream) {
  if (params && !fast_ok(params))
    return nais_train_forward_ex(params, nullptr, hist, n, target, b, dropout_p, seed, pred, saved,
                                 nan_count, workspace, workspace_bytes, stream);
  TShape sh;
  int rc = tvalidate(params, &sh);
  if (rc) return rc;
  if ((rc = check_batch(hist, n, target, b))) return rc;
  if (!(dropout_p >= 0.f && dropout_p <= 1.f))
    return nais_internal_fail(NAIS_E_INVALID, "dropout_p must be in [0, 1]");
  if (b == 0) return NAIS_OK;
  if (!pred || !saved) return nais_internal_fail(NAIS_E_INVALID, "missing pred/saved");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) {  // no history: logit 0 for every row, S = N = 0
    hipLaunchKernelGGL(train_finalize_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, st,
                       nullptr, nullptr, 0, b, n, params->beta, pred, saved, nan_count);
    return nais_internal_check_launch("train_finalize_kernel");
  }
  const int js = slice_items(b, n, FWD_PER_CU);
  const int64_t ns = (n + js - 1) / js;
  if (ns > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "history too long for the grid");
  if (!workspace || workspace_bytes < nais_train_workspace_size(params, b, n))
    return nais_internal_fail(NAIS_E_WORKSPACE, "workspace too small (nais_train_workspace_size)");
  float* Sp = static_cast<float*>(workspace);
  float* Np = Sp + ns * b;
  const TrainArgs a = targs(params, hist, n, target, b, js, dropout_p, seed);
  NAIS_TRAIN_DISPATCH(launch_train_forward, sh, a, Sp, Np, st);
  if (rc) return rc;
  hipLaunchKernelGGL(train_finalize_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, st,
                     Sp, Np, (int)ns, b, n, params->beta, pred, saved, nan_count);
  return nais_internal_check_launch("train_finalize_kernel");
}

int32_t nais_train_backward(const nais_params_t* params, const int64_t* hist, int64_t n,
                            const int64_t* target, int64_t b, float dropout_p, uint64_t seed,
                            const float* pred, const float* saved, const float* grad_pred,
                            float* grad_embed_history, float* grad_embed_target, float* grad_w1,
                            float* grad_b1, float* grad_w2, void* workspace,
                            size_t workspace_bytes, void* stream) {
  if (params && !fast_ok(params)) {
    const nais_train_grads_t g{grad_embed_history, grad_embed_target, nullptr, grad_w1, grad_b1,
                               grad_w2, nullptr, nullptr};
    return nais_train_backward_ex(params, nullptr, hist, n, target, b, dropout_p, seed, pred, saved,
                                  grad_pred, &g, workspace, workspace_bytes, stream);
  }
  TShape sh;
  int rc = tvalidate(params, &sh);
  if (rc) return rc;
  if ((rc = check_batch(hist, n, target, b))) return rc;
  if (!(dropout_p >= 0.f && dropout_p <= 1.f))
    return nais_internal_fail(NAIS_E_INVALID, "dropout_p must be in [0, 1]");
  if (b == 0 || n == 0) return NAIS_OK;  // no history: the logit is constant, all grads 0
  if (!pred || !saved || !grad_pred || !grad_embed_history || !grad_embed_target || !grad_w1 ||
      !grad_b1 || !grad_w2)
    return nais_internal_fail(NAIS_E_INVALID, "missing pred/saved/grad pointer");
  const int js = slice_items(b, n, BWD_PER_CU);
  const int64_t ns = (n + js - 1) / js, rb = (b + TROWS - 1) / TROWS;
  if (ns > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "history too long for the grid");
  if (!workspace || workspace_bytes < nais_train_workspace_size(params, b, n))
    return nais_internal_fail(NAIS_E_WORKSPACE, "workspace too small (nais_train_workspace_size)");
  const int64_t D = params->embed_dim, H = params->hidden;
  float* Wt = static_cast<float*>(workspace);
  float* Ww = Wt + ns * b * D;
  float* Wh = Ww + ns * rb * (H * D + 2 * H);
  const TrainArgs a = targs(params, hist, n, target, b, js, dropout_p, seed);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  NAIS_TRAIN_DISPATCH(launch_train_backward, sh, a, saved, pred, grad_pred, Wt, Ww, Wh, st);
  if (rc) return rc;
  const int64_t total = (H * D + 2 * H) * REDUCE_KS + b * D + n * D;
  hipLaunchKernelGGL(train_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     Wt, Ww, Wh, b, n, (int)D, (int)H, (int)ns, (int)rb, hist, target,
                     grad_embed_history, grad_embed_target, grad_w1, grad_b1, grad_w2, nullptr);
  return nais_internal_check_launch("train_reduce_kernel");
}

int32_t nais_dropout_mask(uint64_t seed, int64_t b, int64_t n, int32_t hidden, float dropout_p,
                          uint8_t* out, void* stream) {
  if (b < 0 || n < 0 || hidden <= 0) return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (!(dropout_p >= 0.f && dropout_p <= 1.f))
    return nais_internal_fail(NAIS_E_INVALID, "dropout_p must be in [0, 1]");
  const int64_t total = b * n * hidden;
  if (total == 0) return NAIS_OK;
  if (!out) return nais_internal_fail(NAIS_E_INVALID, "out is NULL");
  hipLaunchKernelGGL(dropout_mask_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), make_drop(dropout_p, seed), b, n,
                     (int)hidden, out);
  return nais_internal_check_launch("dropout_mask_kernel");
}

int32_t nais_adagrad(float* param, float* state_sum, const float* grad, int64_t numel, float clr,
                     float weight_decay, float eps, void* stream) {
  if (numel < 0) return nais_internal_fail(NAIS_E_INVALID, "negative numel");
  if (numel == 0) return NAIS_OK;
  if (!param || !state_sum || !grad) return nais_internal_fail(NAIS_E_INVALID, "NULL tensor");
  const int64_t blocks = std::min<int64_t>((numel + 255) / 256, 2048 * 4);
  hipLaunchKernelGGL(adagrad_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), param, state_sum, grad, numel, clr,
                     weight_decay, eps);
  return nais_internal_check_launch("adagrad_kernel");
}

int32_t nais_adagrad_rows(float* param, float* state_sum, const float* grad, int32_t dim,
                          const int64_t* rows, int64_t num_rows, float clr, float eps,
                          void* stream) {
  if (num_rows < 0 || dim <= 0) return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (num_rows == 0) return NAIS_OK;
  if (!param || !state_sum || !grad || !rows)
    return nais_internal_fail(NAIS_E_INVALID, "NULL tensor");
  const int64_t total = num_rows * dim;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 2048 * 4);
  hipLaunchKernelGGL(adagrad_rows_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), param, state_sum, grad, dim, rows,
                     num_rows, clr, eps);
  return nais_internal_check_launch("adagrad_rows_kernel");
}


}  // extern "C"
