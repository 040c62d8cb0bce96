// nais_gx.h -- the generic-shape NAIS pair core (not ABI): any embedding width D <= GX_MAX_D and
// any hidden width H, exact fp32 (v_mfma_f32_32x32x2_f32), for the shapes the tuned kernels are
// not compiled for (the reference builds Linear(embed_size, hidden_size) for any sizes,
// model.py:9-38, 100-130, 190-229). Included by nais_generic.hip (scoring: per-user catalog rows,
// pair tables, nais_forward) and nais_train.hip (the training forward / backward at those shapes).
//
// Layout. One wave computes the attention logits of 32 PAIRS at a time: the MFMA columns are 32
// history items (lane & 31) against one target row, the rows 32 hidden units:
//   A (32 x 2)  = W1[32 hb + row][k]       one hidden block of W1 staged in LDS (pitch Q, odd)
//   B (2 x 32)  = x[k][item] = h_item[k] * t[k]   h rows staged in LDS (pitch D + 1, odd; lanes
//                                           over items read distinct banks), t a broadcast row
//   C (32 x 32) = b1 + W1 x  -> ReLU -> . w2 summed into the pair's logit, block by block
// so no operand scales with D or H in registers: W1 is staged one 32-row hidden block at a time
// (the whole W1 would not fit the LDS at D = H = 192), the logit accumulates over the blocks, and
// x is recomputed per block from the LDS rows (one multiply per MFMA). Two targets share every
// A and h read (two independent MFMA chains per wave). K runs over D in steps of 2 (lane half
// hh = lane >> 5 carries k = 2t + hh), then the tail steps: an odd D's last dim and the distance
// variants' 2 features (model.py:265-267, :369-371) as K-step D / D + 1.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nais_internal.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace gx {

__device__ __forceinline__ floatx16 mfma(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// row held in accumulator register r of 32-row block blk by lane half hh (32x32 C layout)
__device__ __forceinline__ int crow(int blk, int r, int hh) {
  return blk * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
}

constexpr int GX_MAX_D = 256;   // the h chunk, the target tile and one W1 block fit the 160 KiB LDS
constexpr int GX_NT = 256;      // threads per workgroup: 4 waves, one per SIMD
constexpr int GX_TT = 32;       // target rows per unit (8 per wave, two MFMA chains at a time)

struct Shape {
  int D, DIN, DINP, Q, HP, H, HB;
  __host__ __device__ Shape(int d, int din, int h)
      : D(d), DIN(din), DINP((din + 1) & ~1), Q(((din + 1) & ~1) + 1), HP(d + 1), H(h),
        HB((h + 31) / 32) {}
};

// W1 rows [32 hb, 32 hb + 32) -> Lw [32][Q] (zero past H rows / DIN columns); b1 -> Lbw[0..32),
// w2 -> Lbw[32..64). Coalesced: consecutive threads read consecutive columns of a row.
__device__ __forceinline__ void stage_w1_block(const float* __restrict__ w1, const float* __restrict__ b1,
                                               const float* __restrict__ w2, const Shape& s, int hb,
                                               float* Lw, float* Lbw, int tid, int nt) {
  for (int r = 0; r < 32; ++r) {
    const int i = 32 * hb + r;
    const float* src = w1 + int64_t(i) * s.DIN;
    for (int k = tid; k < s.Q; k += nt) Lw[r * s.Q + k] = (i < s.H && k < s.DIN) ? src[k] : 0.f;
  }
  if (tid < 64) {
    const int i = 32 * hb + (tid & 31);
    Lbw[tid] = i < s.H ? (tid < 32 ? b1[i] : w2[i]) : 0.f;
  }
}

// One staged hidden block against the 32 items of Lh (rows, pitch s.HP) for up to two target
// rows ta / tb (pitch-free, D floats each; tb ignored unless TWO). fa / fb: the [32][2] distance
// features of the pairs (DIST only). Adds the lane's share of sum_i w2_i relu(z_i) (its 16 rows of
// the block; the other lane half holds the other 16) to pa / pb, and on `first` its share of
// h . t (the dims k == hh mod 2) to sa / sb. drop(k, i): the dropout factor of hidden unit i for
// pair key k (training forward), applied to z before the ReLU as model.py:71 does.
template <bool TWO, bool DIST, bool DROP, typename DF>
__device__ __forceinline__ void block_logits(const Shape& s, const float* __restrict__ Lw,
                                             const float* __restrict__ Lbw, const float* __restrict__ Lh,
                                             const float* __restrict__ ta, const float* __restrict__ tb,
                                             const float* __restrict__ fa, const float* __restrict__ fb,
                                             int lane, int hb, bool first, float& pa, float& pb,
                                             float& sa, float& sb, const DF& drop, uint32_t ka,
                                             uint32_t kb) {
  const int n = lane & 31, hh = lane >> 5;
  floatx16 A, B;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    A[r] = Lbw[crow(0, r, hh)];
    B[r] = A[r];
  }
  const float* hrow = Lh + n * s.HP;
  const float* wrow = Lw + n * s.Q;
  const int D2 = s.D & ~1;
  float xa_s = 0.f, xb_s = 0.f;
#pragma unroll 4
  for (int k0 = 0; k0 < D2; k0 += 2) {
    const int k = k0 + hh;
    const float h = hrow[k], w = wrow[k];
    const float xa = h * ta[k];
    xa_s += xa;
    A = mfma(w, xa, A);
    if (TWO) {
      const float xb = h * tb[k];
      xb_s += xb;
      B = mfma(w, xb, B);
    }
  }
  for (int k0 = D2; k0 < s.DINP; k0 += 2) {   // an odd D's last dim, the distance features
    const int k = k0 + hh;
    float xa = 0.f, xb = 0.f;
    if (k < s.D) {
      const float h = hrow[k];
      xa = h * ta[k];
      xa_s += xa;
      if (TWO) {
        xb = h * tb[k];
        xb_s += xb;
      }
    } else if (DIST && k < s.DIN) {
      xa = fa[2 * n + (k - s.D)];
      if (TWO) xb = fb[2 * n + (k - s.D)];
    }
    A = mfma(wrow[k], xa, A);
    if (TWO) B = mfma(wrow[k], xb, B);
  }
  if (first) {
    sa += xa_s;
    if (TWO) sb += xb_s;
  }
  float qa = 0.f, qb = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = crow(0, r, hh);
    const float w2 = Lbw[32 + i];
    float va = A[r];
    if (DROP) va *= drop(ka, 32 * hb + i);
    qa = fmaf(w2, nais_relu(va), qa);
    if (TWO) {
      float vb = B[r];
      if (DROP) vb *= drop(kb, 32 * hb + i);
      qb = fmaf(w2, nais_relu(vb), qb);
    }
  }
  pa += qa;
  if (TWO) pb += qb;
}

// z = b1 + W1 x of one staged hidden block for one target row t against the 32 items of Lh (C
// layout: lane (n, hh) holds hidden rows crow(0, r, hh) of item n) -- the training backward's
// recompute of the forward (block_logits' arithmetic, one chain)
template <bool DIST>
__device__ __forceinline__ floatx16 block_z(const Shape& s, const float* __restrict__ Lw,
                                            const float* __restrict__ Lbw, const float* __restrict__ Lh,
                                            const float* __restrict__ t, const float* __restrict__ f,
                                            int lane) {
  const int n = lane & 31, hh = lane >> 5;
  floatx16 A;
#pragma unroll
  for (int r = 0; r < 16; ++r) A[r] = Lbw[crow(0, r, hh)];
  const float* hrow = Lh + n * s.HP;
  const float* wrow = Lw + n * s.Q;
  const int D2 = s.D & ~1;
#pragma unroll 4
  for (int k0 = 0; k0 < D2; k0 += 2) {
    const int k = k0 + hh;
    A = mfma(wrow[k], hrow[k] * t[k], A);
  }
  for (int k0 = D2; k0 < s.DINP; k0 += 2) {
    const int k = k0 + hh;
    float x = 0.f;
    if (k < s.D) x = hrow[k] * t[k];
    else if (DIST && k < s.DIN) x = f[2 * n + (k - s.D)];
    A = mfma(wrow[k], x, A);
  }
  return A;
}

struct NoDrop {
  __device__ __forceinline__ float operator()(uint32_t, int) const { return 1.f; }
};

// sum over the 32 lanes of one lane half (every lane of the half gets it)
__device__ __forceinline__ float half_sum32(float v) {
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// sigmoid(dist_layer(scale * ll)) output feature f (model.py:265 / :369), the scorers' op order
__device__ __forceinline__ float dist_feat(const float* wd, const float* bd, float scale, float l0,
                                           float l1, int f) {
  const float m0 = l0 * scale, m1 = l1 * scale;
  return 1.0f / (1.0f + expf(-(m0 * wd[2 * f] + m1 * wd[2 * f + 1] + bd[f])));
}

}  // namespace gx
