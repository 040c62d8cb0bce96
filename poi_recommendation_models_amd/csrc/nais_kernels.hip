// nais_kernels.hip -- MI355X (gfx950 / CDNA4) kernels + C-ABI for the NAIS scoring path.
//
// Reference semantics (muyeon-jo/POI_recommendation_models):
//   attention_network  model.py:57-89 (basic), :144-180 (region), :246-297 (region_distance)
//   mask               model.py:92-95      forward (NaN count + sigmoid) model.py:40-55
//   full-catalog eval  validation.py:11-27, :38-55, :69-127 ; candidates batches.py:52-65
//
// Mapping onto CDNA4. For one (candidate c, history item j) pair the reference evaluates
//   x = h_j (.) t_c ; z = ReLU(W1 x + b1) ; a_j = w2 . z ; e_j = exp(a_j) * [h_j != c]
//   logit_c = sum_j e_j (h_j . t_c) / (sum_j e_j)^beta
// The W1 x products for 32 candidates x 32 hidden units are one v_mfma_f32_32x32x2_f32 per
// K=2 slice (exact fp32 -- a k-ordered fmaf chain, no reduced precision):
//   A (32 x 2)  = W1[i][k]       constant per workgroup, staged once in LDS in fragment order
//   B (2 x 32)  = x[k][c]        formed in VGPRs as t_c[k] * h_j[k]  (t_c lives in VGPRs,
//                                h_j is an LDS broadcast read: every lane of a half reads
//                                the same address)
//   C (32 x 32) = b1[i] + W1 x   lane l holds candidate (l & 31), 16 hidden rows.
// Lane half hh = l >> 5 owns input dims [hh*DH, hh*DH+DH) (DH = D/2); for the region variants
// this is exactly the [item | region] concatenation of model.py:153,157. The ReLU, the w2 dot,
// exp, the beta-smoothed accumulation and h_j . t_c all stay in registers (one xor-32 shuffle
// joins the two lane halves), so nothing of size [b, n, d] or [b, n, H] ever exists in memory.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <string>

#include "nais.h"
#include "nais_internal.h"
#include "nais_geo.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int WAVES = 8;                    // 512-thread workgroups (2 waves per SIMD)
constexpr int THREADS = WAVES * 64;
constexpr int CAND_PER_BLOCK = WAVES * 32;  // one 32-candidate MFMA column tile per wave
constexpr int JC = 64;                      // history rows staged in LDS per chunk
constexpr int TOPK_THREADS = 1024;
constexpr int MAX_K = 1024;
constexpr int MAX_BATCH_USERS = 512;        // users scored per catalog launch
constexpr int PAIR_GROUP_ITEMS = 128;       // item rows per workgroup in pair-table mode

struct DevParams {
  const float* eh;
  const float* et;
  const float* er;
  const float* w1;
  const float* b1;
  const float* w2;
  const float* wd;  // dist_layer.weight [2,2] (region_distance)
  const float* bd;  // dist_layer.bias [2]
  int64_t P;
  int32_t item_dim, region_dim, H, din;
  float beta;
};

// Pair-table mode of the catalog kernels ("pairs" strategy): instead of summing over
// one user's history, a workgroup takes `gi` consecutive rows of an item list (indices[0..nitems))
// and writes, for every (item row r, candidate c) with c in [col0, col0 + cols),
//   e = exp(a) * [item != c]  to e[r * ld + c - col0]   and   e * (h . t)  to es[...]
// -- all a user needs from the pair: pair_gather_kernel sums them over each user's history rows.
// e == nullptr: the normal per-user scoring.
struct TableOut {
  float* e = nullptr;
  float* es = nullptr;
  int64_t ld = 0, col0 = 0, cols = 0, nitems = 0;
  int32_t gi = 0;
  // work queue (x6n only): the launch's item counter, zeroed before it, and the item grid it covers
  int32_t* work = nullptr;
  int32_t ngroups = 0, ntiles = 0;
  // the split16 form (nais_internal.h): e receives the hi words (sel_e = NAIS_SEL_HI, one
  // v_perm_b32), es the exact (e, e*s) pairs with row pitch 2 * ld (ex = 1)
  uint32_t sel_e = NAIS_SEL_E;
  int32_t ex = 0;
};
// the pair's two terms for item row `row` (relative to the launch's base) and column offset x
__device__ __forceinline__ void tab_put(const TableOut& t, int64_t row, int64_t x, float e, float es) {
  const int64_t o = row * t.ld + x;
  const uint32_t eb = __float_as_uint(e), sb = __float_as_uint(es);
  t.e[o] = __uint_as_float(__builtin_amdgcn_perm(sb, eb, t.sel_e));
  if (t.ex) {
    reinterpret_cast<float2*>(t.es)[o] = make_float2(e, es);
  } else {
    t.es[o] = es;
  }
}

// Catalog grid: one workgroup per (user slot, 256-POI tile), user-major dispatch order
// (blockIdx.x = tile): a user's ~400 workgroups run back to back, heaviest users first. (A
// tile-major order that keeps the 64 KB of target rows per tile in one XCD's L2 measured slower:
// fp32 -11 %, fp16x3 -3 %, profiles/r1/ab_tilemajor.json -- the kernel is MFMA-bound and the
// Infinity Cache serves the re-reads far below any limit.)
__device__ __forceinline__ int cat_user_slot() { return blockIdx.y; }
__device__ __forceinline__ int cat_tile() { return blockIdx.x; }
inline dim3 table_grid(const TableOut& t, int ngroups, int cand_per_block = CAND_PER_BLOCK) {
  return dim3((unsigned)((t.cols + cand_per_block - 1) / cand_per_block), (unsigned)ngroups);
}
inline dim3 cat_grid(int64_t P, int nb, int cand_per_block) {
  return dim3((unsigned)((P + cand_per_block - 1) / cand_per_block), (unsigned)nb);
}

// What each variant carries: the region half of the concatenation (model.py:153,157) and the
// 2-feature distance input (model.py:265-267 at x100, model.py:369-371 at x1000).
template <int VAR>
struct VarT {
  static constexpr bool REGION = VAR == NAIS_VARIANT_REGION || VAR == NAIS_VARIANT_REGION_DISTANCE;
  static constexpr bool DIST = VAR == NAIS_VARIANT_REGION_DISTANCE || VAR == NAIS_VARIANT_DISTANCE;
  static constexpr float DSCALE = VAR == NAIS_VARIANT_DISTANCE ? 1000.f : 100.f;
};

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---------------------------------------------------------------------------------------------
// Workgroup-constant operands: W1 in MFMA-A fragment order, b1/w2 in accumulator-row order.
// ---------------------------------------------------------------------------------------------
template <int DH, int HB, bool DIST>
struct Consts {
  static constexpr int A4 = HB * (DH / 4) * 64;  // float4 entries of the W1 image
  static constexpr int ADIST = DIST ? HB * 64 : 0;
  static constexpr int EPI = 2 * 2 * HB * 16;    // b1 then w2, each [hh][hb*16+r]
  static constexpr size_t BYTES = size_t(A4) * 16 + size_t(ADIST) * 4 + size_t(EPI) * 4;
};

// hidden row held in accumulator register r of block hb by lane half hh (32x32 C layout)
__device__ __forceinline__ int acc_row(int hb, int r, int hh) {
  return hb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
}

template <int DH, int HB, bool DIST>
__device__ void stage_consts(const DevParams& p, float4* Aimg, float* Adist, float* Eimg, int tid) {
  using C = Consts<DH, HB, DIST>;
  constexpr int D = 2 * DH;
  for (int f = tid; f < C::A4; f += THREADS) {
    const int ln = f & 63, q = (f >> 6) % (DH / 4), hb = (f >> 6) / (DH / 4);
    const int i = hb * 32 + (ln & 31), k0 = (ln >> 5) * DH + 4 * q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < p.H) {
      const float* w = p.w1 + (int64_t)i * p.din + k0;
      v = make_float4(w[0], w[1], w[2], w[3]);
    }
    Aimg[f] = v;
  }
  if (DIST) {
    for (int f = tid; f < C::ADIST; f += THREADS) {
      const int ln = f & 63, hb = f >> 6, i = hb * 32 + (ln & 31);
      Adist[f] = (i < p.H) ? p.w1[(int64_t)i * p.din + D + (ln >> 5)] : 0.f;
    }
  }
  for (int f = tid; f < C::EPI; f += THREADS) {
    const int which = f / (2 * HB * 16), rem = f % (2 * HB * 16);
    const int hh = rem / (HB * 16), hr = rem % (HB * 16), hb = hr / 16, r = hr % 16;
    const int i = acc_row(hb, r, hh);
    Eimg[f] = (i < p.H) ? (which == 0 ? p.b1[i] : p.w2[i]) : 0.f;
  }
}

// One history item j against the lane's candidate: returns a_j (attn_layer2 output) and
// s_j = h_j . t_c, both already combined across the two lane halves.
//   hrow: this lane-half's DH floats of h_j (LDS broadcast or per-lane global)
template <int DH, int HB, bool DIST, typename HPtr, typename EpiT>
__device__ __forceinline__ void item_step(const float4 (&t4)[DH / 4], HPtr hrow,
                                          const float4* __restrict__ Aimg,
                                          const float* __restrict__ Adist, const EpiT& epi,
                                          float distf, int lane, float& a_out, float& s_out) {
  // hidden blocks in passes of at most 4 (128 hidden units): more than 4 blocks' accumulators
  // (H > 128) would not fit the VGPRs beside t and h; x = t * h is recomputed per pass
  constexpr int HS = HB > 4 ? 4 : HB;
  float sd = 0.f, ap = 0.f;
#pragma unroll 1
  for (int h0 = 0; h0 < HB; h0 += HS) {
    floatx16 acc[HS];
#pragma unroll
    for (int hb = 0; hb < HS; ++hb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[hb][r] = epi.bias((h0 + hb) * 16 + r);
    // Software pipeline over the DH/4 k-groups: the LDS operands of group q+1 are requested before
    // the 4*HS MFMAs of group q issue; sched_barrier keeps the compiler from hoisting every load of
    // the item to the top (which costs ~HS*DH VGPRs and spills at D = H = 128).
    float4 hv_n = *reinterpret_cast<const float4*>(hrow);
    float4 a_n[HS];
#pragma unroll
    for (int hb = 0; hb < HS; ++hb) a_n[hb] = Aimg[((h0 + hb) * (DH / 4)) * 64 + lane];
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) {
      const float4 hv = hv_n;
      float4 a_c[HS];
#pragma unroll
      for (int hb = 0; hb < HS; ++hb) a_c[hb] = a_n[hb];
      if (q + 1 < DH / 4) {
        hv_n = *reinterpret_cast<const float4*>(hrow + 4 * (q + 1));
#pragma unroll
        for (int hb = 0; hb < HS; ++hb) a_n[hb] = Aimg[((h0 + hb) * (DH / 4) + q + 1) * 64 + lane];
      }
      const float x0 = t4[q].x * hv.x, x1 = t4[q].y * hv.y, x2 = t4[q].z * hv.z, x3 = t4[q].w * hv.w;
      if (h0 == 0) {
        sd += x0;
        sd += x1;
        sd += x2;
        sd += x3;
      }
#pragma unroll
      for (int hb = 0; hb < HS; ++hb) {
        acc[hb] = mfma32(a_c[hb].x, x0, acc[hb]);
        acc[hb] = mfma32(a_c[hb].y, x1, acc[hb]);
        acc[hb] = mfma32(a_c[hb].z, x2, acc[hb]);
        acc[hb] = mfma32(a_c[hb].w, x3, acc[hb]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (DIST) {
#pragma unroll
      for (int hb = 0; hb < HS; ++hb) acc[hb] = mfma32(Adist[(h0 + hb) * 64 + lane], distf, acc[hb]);
    }
#pragma unroll
    for (int hb = 0; hb < HS; ++hb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[hb][r];
        const float z = (v < 0.f) ? 0.f : v;  // ReLU that keeps NaN, as torch.relu
        ap = __builtin_fmaf(epi.w2((h0 + hb) * 16 + r), z, ap);
      }
  }
  a_out = ap + __shfl_xor(ap, 32);
  s_out = sd + __shfl_xor(sd, 32);
}

// region_distance feature of one (c, j) pair for lane half hh (model.py:265; the pair's
// (|dlat|, |dlng|) is formed in float64 and cast to float32 as at run.py:51-52 / validation.py:118)
struct DistW {
  float w0, w1, b;  // row hh of dist_layer: this lane half computes output feature hh
  float scale;      // the variant's input scale (x100 / x1000)
};
template <int VAR>
__device__ __forceinline__ DistW load_distw(const DevParams& p, int hh) {
  return DistW{p.wd[2 * hh], p.wd[2 * hh + 1], p.bd[hh], VarT<VAR>::DSCALE};
}
__device__ __forceinline__ float dist_feature(const DistW& w, float ll0, float ll1) {
  const float m0 = ll0 * w.scale, m1 = ll1 * w.scale;
  return sigmoidf_ref(m0 * w.w0 + m1 * w.w1 + w.b);
}

// b1 / w2 for this lane half's accumulator rows: in VGPRs for H <= 64, else read from the LDS
// image at each use (keeps H = 128 within the 256-VGPR budget of 2 waves per SIMD).
template <int HB, bool REGS>
struct Epi;
template <int HB>
struct Epi<HB, true> {
  float b[HB * 16], w[HB * 16];
  __device__ __forceinline__ void load(const float* Eimg, int hh) {
#pragma unroll
    for (int i = 0; i < HB * 16; ++i) {
      b[i] = Eimg[hh * HB * 16 + i];
      w[i] = Eimg[2 * HB * 16 + hh * HB * 16 + i];
    }
  }
  __device__ __forceinline__ float bias(int i) const { return b[i]; }
  __device__ __forceinline__ float w2(int i) const { return w[i]; }
};
template <int HB>
struct Epi<HB, false> {
  const float* pb;
  const float* pw;
  __device__ __forceinline__ void load(const float* Eimg, int hh) {
    pb = Eimg + hh * HB * 16;
    pw = Eimg + 2 * HB * 16 + hh * HB * 16;
  }
  __device__ __forceinline__ float bias(int i) const { return pb[i]; }
  __device__ __forceinline__ float w2(int i) const { return pw[i]; }
};

__device__ __forceinline__ float finish_logit(float S, float N, float beta, bool empty) {
  if (empty) return 0.f;  // sum over an empty history dim (model.py:79-88 with n == 0)
  const float den = (beta == 0.5f) ? sqrtf(S) : powf(S, beta);
  return N / den;
}

// ---------------------------------------------------------------------------------------------
// Full-catalog scoring: grid (ceil(P / 256), users in batch). Each workgroup = one user x 256
// consecutive POI ids; the user's history rows are staged into LDS once per 64-row chunk and
// broadcast to all 8 waves. Scores of history POIs are written as -1 (excluded from top-k).
// ---------------------------------------------------------------------------------------------
template <int DH, int HB, int VAR>
__global__ void __launch_bounds__(THREADS, 1)
catalog_score_kernel(DevParams p, const int64_t* __restrict__ indptr,
                     const int64_t* __restrict__ indices, const int32_t* __restrict__ users,
                     const int64_t* __restrict__ region_of, const double* __restrict__ coords,
                     const double* __restrict__ latlon_mat, float* __restrict__ scores,
                     int64_t score_ld, int32_t* __restrict__ nan_count, TableOut tab) {
  constexpr bool REGION = VarT<VAR>::REGION;
  constexpr bool DIST = VarT<VAR>::DIST;
  constexpr int D = 2 * DH;
  using C = Consts<DH, HB, DIST>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* Aimg = reinterpret_cast<float4*>(smem);
  float* Adist = reinterpret_cast<float*>(Aimg + C::A4);
  float* Eimg = Adist + C::ADIST;
  float* hrows = Eimg + C::EPI;
  int32_t* hid = reinterpret_cast<int32_t*>(hrows + JC * D);
  double* hco = reinterpret_cast<double*>(hid + JC);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
  int64_t hbeg, hlen;
  if (tab.e) {   // pair-table mode: a group of tab.gi rows of the item list
    hbeg = (int64_t)cat_user_slot() * tab.gi;
    hlen = std::min<int64_t>(tab.gi, tab.nitems - hbeg);
  } else {
    const int64_t u = users[cat_user_slot()];
    hbeg = indptr[u];
    hlen = indptr[u + 1] - hbeg;
  }
  const int64_t c = tab.col0 + (int64_t)cat_tile() * CAND_PER_BLOCK + wave * 32 + (lane & 31);
  const bool valid = c < p.P && (!tab.e || c < tab.col0 + tab.cols);
  const int64_t cc = valid ? c : p.P - 1;

  stage_consts<DH, HB, DIST>(p, Aimg, Adist, Eimg, tid);

  // candidate operand: t_c (this lane half's DH dims) in VGPRs for the whole history sweep
  float4 t4[DH / 4];
  {
    const float* src = (REGION && hh) ? p.er + region_of[cc] * p.region_dim
                                      : p.et + cc * p.item_dim + (REGION ? 0 : hh * DH);
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) t4[q] = reinterpret_cast<const float4*>(src)[q];
  }
  double clat = 0.0, clon = 0.0;
  DistW dw{0.f, 0.f, 0.f};
  const double* llrow = nullptr;  // latlon_mat row of this candidate (matrix mode)
  if (DIST) {
    if (coords) {
      clat = coords[2 * cc];
      clon = coords[2 * cc + 1];
    } else {
      llrow = latlon_mat + cc * p.P * 2;
    }
    dw = load_distw<VAR>(p, hh);
  }

  float S = 0.f, N = 0.f;
  bool in_hist = false;
  Epi<HB, (HB <= 2 && DH <= 32)> epi;
  __syncthreads();
  epi.load(Eimg, hh);

  for (int64_t j0 = 0; j0 < hlen; j0 += JC) {
    const int jn = (int)std::min<int64_t>(JC, hlen - j0);
    __syncthreads();  // consumers of the previous chunk are done
    for (int f = tid; f < jn * (D / 4); f += THREADS) {
      const int jj = f / (D / 4), q4 = f % (D / 4);
      const int64_t item = indices[hbeg + j0 + jj];
      float4 v;
      if (!REGION || q4 < DH / 4)
        v = reinterpret_cast<const float4*>(p.eh + item * p.item_dim)[q4];
      else
        v = reinterpret_cast<const float4*>(p.er + region_of[item] * p.region_dim)[q4 - DH / 4];
      reinterpret_cast<float4*>(hrows)[f] = v;
    }
    for (int jj = tid; jj < jn; jj += THREADS) {
      const int64_t item = indices[hbeg + j0 + jj];
      hid[jj] = (int32_t)item;
      if (DIST && coords) {
        hco[2 * jj] = coords[2 * item];
        hco[2 * jj + 1] = coords[2 * item + 1];
      }
    }
    __syncthreads();
    for (int jj = 0; jj < jn; ++jj) {
      float distf = 0.f;
      if (DIST) {
        float ll0, ll1;
        if (coords) {
          ll0 = (float)fabs(clat - hco[2 * jj]);
          ll1 = (float)fabs(clon - hco[2 * jj + 1]);
        } else {
          ll0 = (float)llrow[2 * (int64_t)hid[jj]];
          ll1 = (float)llrow[2 * (int64_t)hid[jj] + 1];
        }
        distf = dist_feature(dw, ll0, ll1);
      }
      float a, s;
      item_step<DH, HB, DIST>(t4, hrows + jj * D + hh * DH, Aimg, Adist, epi, distf, lane, a, s);
      const bool keep = hid[jj] != (int32_t)c;             // model.py:92-95
      const float e = expf(a) * (keep ? 1.f : 0.f);        // model.py:75-78 (inf * 0 -> NaN)
      if (tab.e) {
        if (valid && hh == 0) {
          tab_put(tab, hbeg + j0 + jj, c - tab.col0, e, e * s);
        }
        continue;
      }
      in_hist |= !keep;
      S += e;                                               // model.py:79
      N += e * s;                                           // sum_j w_j (h_j . t) numerator
    }
  }
  if (tab.e) return;

  const float logit = finish_logit(S, N, p.beta, hlen == 0);
  const bool isnan_ = logit != logit;
  float sc = sigmoidf_ref(logit);
  if (isnan_) sc = __builtin_nanf("");
  if (in_hist) sc = -1.f;  // history POI: not a candidate (batches.py:56)
  if (valid && hh == 0) scores[(int64_t)cat_user_slot() * score_ld + c] = sc;
  if (nan_count) {
    const unsigned long long m = __ballot(valid && hh == 0 && !in_hist && isnan_);
    if (lane == 0 && m) atomicAdd(nan_count, (int32_t)__popcll(m));
  }
}

// ---------------------------------------------------------------------------------------------
// General forward: arbitrary per-row histories; each lane gathers its own row's h_j from
// global memory (L2/MALL-resident tables), one item ahead of the MFMA sweep.
// ---------------------------------------------------------------------------------------------
template <int DH, int HB, int VAR>
__global__ void __launch_bounds__(THREADS, 1)
forward_kernel(DevParams p, const int64_t* __restrict__ hist, int64_t b, int64_t n, int64_t hist_ld,
               const int64_t* __restrict__ target, const int64_t* __restrict__ hist_region,
               int64_t hreg_ld, const int64_t* __restrict__ target_region,
               const float* __restrict__ latlon, int64_t ll_ld, float* __restrict__ out,
               int32_t* __restrict__ nan_count, int32_t flags) {
  constexpr bool REGION = VarT<VAR>::REGION;
  constexpr bool DIST = VarT<VAR>::DIST;
  using C = Consts<DH, HB, DIST>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float4* Aimg = reinterpret_cast<float4*>(smem);
  float* Adist = reinterpret_cast<float*>(Aimg + C::A4);
  float* Eimg = Adist + C::ADIST;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
  const int64_t r = (int64_t)blockIdx.x * CAND_PER_BLOCK + wave * 32 + (lane & 31);
  const bool valid = r < b;
  const int64_t rr = valid ? r : b - 1;
  stage_consts<DH, HB, DIST>(p, Aimg, Adist, Eimg, tid);

  const int64_t tgt = target[rr];
  float4 t4[DH / 4];
  {
    const float* src = (REGION && hh) ? p.er + target_region[rr] * p.region_dim
                                      : p.et + tgt * p.item_dim + (REGION ? 0 : hh * DH);
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) t4[q] = reinterpret_cast<const float4*>(src)[q];
  }
  const int64_t* hrow_ids = hist + rr * hist_ld;
  DistW dw{0.f, 0.f, 0.f};
  if (DIST) dw = load_distw<VAR>(p, hh);
  auto row_ptr = [&](int64_t j) -> const float* {
    const int64_t item = hrow_ids[j];
    if (REGION && hh) return p.er + hist_region[rr * hreg_ld + j] * p.region_dim;
    return p.eh + item * p.item_dim + (REGION ? 0 : hh * DH);
  };

  Epi<HB, (HB <= 2 && DH <= 32)> epi;
  __syncthreads();
  epi.load(Eimg, hh);

  float S = 0.f, N = 0.f;
  constexpr bool PREFETCH = DH <= 32;  // one-item-ahead gather; at D = 128 it would spill
  float4 hcur[DH / 4];
  if (PREFETCH && n > 0) {
    const float* hp = row_ptr(0);
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) hcur[q] = reinterpret_cast<const float4*>(hp)[q];
  }
  for (int64_t j = 0; j < n; ++j) {
    float4 hnext[DH / 4];
    if (!PREFETCH) {
      const float* hp = row_ptr(j);
#pragma unroll
      for (int q = 0; q < DH / 4; ++q) hcur[q] = reinterpret_cast<const float4*>(hp)[q];
    } else if (j + 1 < n) {
      const float* hp = row_ptr(j + 1);
#pragma unroll
      for (int q = 0; q < DH / 4; ++q) hnext[q] = reinterpret_cast<const float4*>(hp)[q];
    }
    float distf = 0.f;
    if (DIST) {
      const float* ll = latlon + rr * ll_ld + 2 * j;
      distf = dist_feature(dw, ll[0], ll[1]);
    }
    float a, s;
    item_step<DH, HB, DIST>(t4, reinterpret_cast<const float*>(hcur), Aimg, Adist, epi, distf,
                            lane, a, s);
    const bool keep = hrow_ids[j] != tgt;
    const float e = expf(a) * (keep ? 1.f : 0.f);
    S += e;
    N += e * s;
    if (PREFETCH && j + 1 < n) {
#pragma unroll
      for (int q = 0; q < DH / 4; ++q) hcur[q] = hnext[q];
    }
  }
  const float logit = finish_logit(S, N, p.beta, n == 0);
  const bool isnan_ = logit != logit;
  float o = (flags & NAIS_FLAG_SIGMOID) ? sigmoidf_ref(logit) : logit;
  if (valid && hh == 0) out[r] = o;
  if (nan_count) {
    const unsigned long long m = __ballot(valid && hh == 0 && isnan_);
    if (lane == 0 && m) atomicAdd(nan_count, (int32_t)__popcll(m));
  }
}

// ---------------------------------------------------------------------------------------------
// Split-fp16 ("3xf16") catalog scorer: the same computation as catalog_score_kernel with the
// W1 x products on v_mfma_f32_32x32x16_f16 (16x the f32-MFMA rate). Every fp32 operand v is
// scaled by a power of two (exact) into fp16 range and split v = hi + lo, hi = f16(v),
// lo = f16(v - hi) (22 significant bits together); the product is accumulated in fp32 as
//   al*bh + ah*bl + ah*bh        (al*bl ~ 2^-22 relative is dropped),
// i.e. ~2^-21 relative per product against fp32's 2^-24 -- scores stay within ~2e-7 of the
// reference (tests/test_gpu_parity.py, both precisions). Scales:
//   S_w = 2^e: max|W1[:, :D]| * S_w in [2^13, 2^14)   (per workgroup, from the LDS image)
//   S_t = 2^e per candidate and history chunk: max|t_c| * max|h_chunk| * S_t in [2^13, 2^14),
//         applied to t_c (so x_s = t_s * h_j = S_t * fl32(t_c * h_j) exactly).
// b1 / w2 are pre-scaled per chunk so acc = S_w*S_t*(W1 x + b1) and a_j = sum w2/(S_w S_t) relu(acc).
// ---------------------------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ floatx16 mfma16(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// 2^e with m * 2^e in [2^13, 2^14) for finite m > 0 (clamped), 1 otherwise
__device__ __forceinline__ float pow2_scale(float m) {
  if (!(m > 0.f) || !(m < __builtin_huge_valf())) return 1.f;
  const uint32_t bits = __float_as_uint(m);
  int ex = (int)((bits >> 23) & 255u) - 127;
  if (((bits >> 23) & 255u) == 0u) ex = -127;  // subnormal product: maximal (clamped) scale
  int e = 13 - ex;
  e = e < -120 ? -120 : (e > 120 ? 120 : e);
  return __uint_as_float((uint32_t)(e + 127) << 23);
}

// x -> (hi, lo): hi = f16(x) (RNE, v_cvt_pk_f16_f32), lo = f16(x - hi) with the subtraction done
// exactly inside v_fma_mix{lo,hi}_f16 (one instruction per element instead of cvt + sub + cvt).
// The trailing s_nop 1 covers the VALU-write -> MFMA-operand-read hazard that hipcc does not
// pad for inline asm (cdna_hip_programming.md 5.7 item 2).
__device__ __forceinline__ void split8(const float (&x)[8], half8& hi, half8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) hi[e] = (_Float16)x[e];
  const uint4 hu = *reinterpret_cast<const uint4*>(&hi);
  uint32_t l0, l1, l2, l3;
  asm("v_fma_mixlo_f16 %0, -%4, 1.0, %8 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, -%4, 1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %1, -%5, 1.0, %10 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, -%5, 1.0, %11 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %2, -%6, 1.0, %12 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %2, -%6, 1.0, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %3, -%7, 1.0, %14 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %3, -%7, 1.0, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "s_nop 1"
      : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
      : "v"(hu.x), "v"(hu.y), "v"(hu.z), "v"(hu.w), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]),
        "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]));
  const uint4 lu = make_uint4(l0, l1, l2, l3);
  lo = *reinterpret_cast<const half8*>(&lu);
}

// x -> (hi, mid, lo), x == hi + mid + lo exactly for the scaled operands of this file (33
// significant bits >= fp32's 24; f16 subnormals only below 2^-37 of the scaled maximum):
//   hi = f16(x),  r = x - hi (exact, v_fma_mix_f32),  mid = f16(r),  lo = f16(r - mid) (exact
//   subtraction inside v_fma_mix{lo,hi}_f16). The fp16x6 path multiplies such splits (6 products).
__device__ __forceinline__ void split8_3(const float (&x)[8], half8& hi, half8& mid, half8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) hi[e] = (_Float16)x[e];
  const uint4 hu = *reinterpret_cast<const uint4*>(&hi);
  const uint32_t hw[4] = {hu.x, hu.y, hu.z, hu.w};
  float r[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    asm("v_fma_mix_f32 %0, -%2, 1.0, %3 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mix_f32 %1, -%2, 1.0, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(r[2 * q]), "=&v"(r[2 * q + 1])
        : "v"(hw[q]), "v"(x[2 * q]), "v"(x[2 * q + 1]));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) mid[e] = (_Float16)r[e];
  const uint4 mu = *reinterpret_cast<const uint4*>(&mid);
  uint32_t l0, l1, l2, l3;
  asm("v_fma_mixlo_f16 %0, -%4, 1.0, %8 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, -%4, 1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %1, -%5, 1.0, %10 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, -%5, 1.0, %11 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %2, -%6, 1.0, %12 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %2, -%6, 1.0, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %3, -%7, 1.0, %14 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %3, -%7, 1.0, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "s_nop 1"
      : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
      : "v"(mu.x), "v"(mu.y), "v"(mu.z), "v"(mu.w), "v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]),
        "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7]));
  const uint4 lu = make_uint4(l0, l1, l2, l3);
  lo = *reinterpret_cast<const half8*>(&lu);
}

// NPC split pieces of 8 fp32 values: 2 = (hi, lo) for fp16x3, 3 = (hi, mid, lo) for fp16x6
template <int NPC>
__device__ __forceinline__ void split_pieces(const float (&x)[8], half8 (&pc)[NPC]) {
  if constexpr (NPC == 2) split8(x, pc[0], pc[1]);
  else split8_3(x, pc[0], pc[1], pc[2]);
}

// c += a . b over the pieces, smallest terms first:
//   NPC = 2 (fp16x3): al*bh + ah*bl + ah*bh       -- al*bl (~2^-22 relative) dropped
//   NPC = 3 (fp16x6): the six terms of order <= 2^-22 (lo*hi, mid*mid, hi*lo, mid*hi, hi*mid,
//                     hi*hi); the dropped mid*lo, lo*mid, lo*lo are <= ~2^-33 relative, below
//                     fp32's own 2^-24 rounding of the product -- fp32-faithful products.
template <int NPC>
__device__ __forceinline__ floatx16 mfma_pieces(const half8 (&a)[NPC], const half8 (&b)[NPC], floatx16 c) {
  if constexpr (NPC == 2) {
    c = mfma16(a[1], b[0], c);
    c = mfma16(a[0], b[1], c);
    c = mfma16(a[0], b[0], c);
  } else {
    c = mfma16(a[2], b[0], c);
    c = mfma16(a[1], b[1], c);
    c = mfma16(a[0], b[2], c);
    c = mfma16(a[1], b[0], c);
    c = mfma16(a[0], b[1], c);
    c = mfma16(a[0], b[0], c);
  }
  return c;
}

// Both lane halves' values of v in every lane, by one v_permlane32_swap (VALU, no LDS):
// .x = v[lane & 31], .y = v[32 + (lane & 31)]; .x + .y == v + shfl_xor(v, 32) exactly.
__device__ __forceinline__ float2 lane_halves(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return make_float2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

template <int NW>
__device__ float block_max_n(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
  return m;
}

__device__ float block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int w = 1; w < WAVES; ++w) m = fmaxf(m, red[w]);
  return m;
}

template <int DH, int HB, bool DIST, int NPC = 2>
struct Consts16 {
  static constexpr int KS = DH / 8;                 // f16 MFMA K-steps (8 dims per lane half)
  static constexpr int A16 = HB * KS * NPC * 64;    // uint4 entries: [hb][s][piece][lane]
  static constexpr int ADIST = DIST ? HB * 64 : 0;  // fp32 (S_w-scaled) distance columns
  static constexpr int EPI = 2 * 2 * HB * 16;
  static constexpr size_t BYTES = size_t(A16) * 16 + size_t(ADIST) * 4 + size_t(EPI) * 4 + 64;
};

// ReLU that keeps every NaN, as torch.relu (model.py:71): gfx950's v_maximum3_f32 (IEEE 754-2019
// maximum: NaN propagates, max(-0, +0) = +0), one VALU. (The round-2 form, v_cmp + v_cndmask on
// the float bits, was 1.1 % slower on the pair table: profiles/r3/relu_ab.)
__device__ __forceinline__ float relu_bits(float v) {
  return __builtin_elementwise_maximum(v, 0.f);   // v_maximum3_f32: IEEE maximum, NaN in -> NaN out
}

template <int HB, bool REGS>
struct Epi16;
template <int HB>
struct Epi16<HB, true> {           // pre-scaled copies in VGPRs: acc starts at S*b1
  float bs[HB * 16], ws[HB * 16];
  __device__ __forceinline__ void rescale(const float* Eimg, int hh, float S, float invS) {
#pragma unroll
    for (int i = 0; i < HB * 16; ++i) {
      bs[i] = Eimg[hh * HB * 16 + i] * S;
      ws[i] = Eimg[2 * HB * 16 + hh * HB * 16 + i] * invS;
    }
  }
  __device__ __forceinline__ float init(int i) const { return bs[i]; }
  __device__ __forceinline__ float term(int i, float acc, float) const {
    return ws[i] * relu_bits(acc);
  }
};
template <int HB>
struct Epi16<HB, false> {          // b1 / w2 read from LDS: acc starts at 0, unscaled per use
  const float* pb;
  const float* pw;
  __device__ __forceinline__ void rescale(const float* Eimg, int hh, float, float) {
    pb = Eimg + hh * HB * 16;
    pw = Eimg + 2 * HB * 16 + hh * HB * 16;
  }
  __device__ __forceinline__ float init(int) const { return 0.f; }
  __device__ __forceinline__ float term(int i, float acc, float invS) const {
    return pw[i] * relu_bits(__builtin_fmaf(acc, invS, pb[i]));
  }
};

template <int HB>
struct Epi16L {                    // per-wave LDS copy of S*b1 and w2/S (S wave-uniform): acc starts at S*b1
  const float* pb;
  const float* pw;
  __device__ __forceinline__ void rescale(const float* mine, int hh, float, float) {
    pb = mine + hh * HB * 16;
    pw = mine + 2 * HB * 16 + hh * HB * 16;
  }
  __device__ __forceinline__ float init(int i) const { return pb[i]; }
  __device__ __forceinline__ float term(int i, float acc, float) const {
    return pw[i] * relu_bits(acc);
  }
};

template <int DH, int HB, int VAR, int NPC>
__global__ void __launch_bounds__(THREADS, 1)
catalog_score_x3_kernel(DevParams p, const int64_t* __restrict__ indptr,
                        const int64_t* __restrict__ indices, const int32_t* __restrict__ users,
                        const int64_t* __restrict__ region_of, const double* __restrict__ coords,
                        const double* __restrict__ latlon_mat, float* __restrict__ scores,
                        int64_t score_ld, int32_t* __restrict__ nan_count, TableOut tab) {
  constexpr bool REGION = VarT<VAR>::REGION;
  constexpr bool DIST = VarT<VAR>::DIST;
  constexpr int D = 2 * DH;
  constexpr int KS = DH / 8;
  constexpr bool EREGS = HB <= 2 && DH <= 32;
  // one-step-ahead fragment prefetch only where the registers allow it
  constexpr bool PREF = NPC == 2 && HB <= 2;
  using C = Consts16<DH, HB, DIST, NPC>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* A16 = reinterpret_cast<uint4*>(smem);
  float* Adist = reinterpret_cast<float*>(A16 + C::A16);
  float* Eimg = Adist + C::ADIST;
  float* red = Eimg + C::EPI;                        // 16 floats of reduction scratch
  float* hrows = red + 16;
  int32_t* hid = reinterpret_cast<int32_t*>(hrows + JC * D);
  double* hco = reinterpret_cast<double*>(hid + JC);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
  int64_t hbeg, hlen;
  if (tab.e) {   // pair-table mode: a group of tab.gi rows of the item list
    hbeg = (int64_t)cat_user_slot() * tab.gi;
    hlen = std::min<int64_t>(tab.gi, tab.nitems - hbeg);
  } else {
    const int64_t u = users[cat_user_slot()];
    hbeg = indptr[u];
    hlen = indptr[u + 1] - hbeg;
  }
  const int64_t c = tab.col0 + (int64_t)cat_tile() * CAND_PER_BLOCK + wave * 32 + (lane & 31);
  const bool valid = c < p.P && (!tab.e || c < tab.col0 + tab.cols);
  const int64_t cc = valid ? c : p.P - 1;

  // ---- W1 scale, then the split A image (hi/lo per 8-dim slice) and the fp32 distance columns
  float wmax = 0.f;
  for (int f = tid; f < p.H * D; f += THREADS) {
    const int i = f / D, k = f - i * D;
    wmax = fmaxf(wmax, fabsf(p.w1[(int64_t)i * p.din + k]));
  }
  const float Sw = pow2_scale(block_max(wmax, red));
  for (int f = tid; f < C::A16; f += THREADS) {
    const int ln = f & 63, part = (f >> 6) % NPC, s = ((f >> 6) / NPC) % KS, hb = ((f >> 6) / NPC) / KS;
    const int i = hb * 32 + (ln & 31), k0 = (ln >> 5) * DH + 8 * s;
    half8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float w = (i < p.H) ? p.w1[(int64_t)i * p.din + k0 + e] * Sw : 0.f;
      const _Float16 hi = (_Float16)w;
      const float r = w - (float)hi;                  // exact
      const _Float16 mid = (_Float16)r;
      v[e] = part == 0 ? hi : (part == 1 ? mid : (_Float16)(r - (float)mid));
    }
    A16[f] = *reinterpret_cast<const uint4*>(&v);
  }
  if (DIST) {
    for (int f = tid; f < C::ADIST; f += THREADS) {
      const int ln = f & 63, hb = f >> 6, i = hb * 32 + (ln & 31);
      Adist[f] = (i < p.H) ? p.w1[(int64_t)i * p.din + D + (ln >> 5)] * Sw : 0.f;
    }
  }
  for (int f = tid; f < C::EPI; f += THREADS) {
    const int which = f / (2 * HB * 16), rem = f % (2 * HB * 16);
    const int hh2 = rem / (HB * 16), hr = rem % (HB * 16), hb = hr / 16, r = hr % 16;
    const int i = acc_row(hb, r, hh2);
    Eimg[f] = (i < p.H) ? (which == 0 ? p.b1[i] : p.w2[i]) : 0.f;
  }

  // ---- candidate operand t_c (fp32, this lane half's DH dims) and its max magnitude
  float tv[DH];
  {
    const float* src = (REGION && hh) ? p.er + region_of[cc] * p.region_dim
                                      : p.et + cc * p.item_dim + (REGION ? 0 : hh * DH);
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(src)[q];
      tv[4 * q] = v.x;
      tv[4 * q + 1] = v.y;
      tv[4 * q + 2] = v.z;
      tv[4 * q + 3] = v.w;
    }
  }
  float tmax = 0.f;
#pragma unroll
  for (int k = 0; k < DH; ++k) tmax = fmaxf(tmax, fabsf(tv[k]));
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
  double clat = 0.0, clon = 0.0;
  DistW dw{0.f, 0.f, 0.f};
  const double* llrow = nullptr;
  if (DIST) {
    if (coords) {
      clat = coords[2 * cc];
      clon = coords[2 * cc + 1];
    } else {
      llrow = latlon_mat + cc * p.P * 2;
    }
    dw = load_distw<VAR>(p, hh);
  }

  float S = 0.f, N = 0.f;
  bool in_hist = false;
  float St = 1.f;                      // current scale applied to tv[]
  Epi16<HB, EREGS> epi;

  for (int64_t j0 = 0; j0 < hlen; j0 += JC) {
    const int jn = (int)std::min<int64_t>(JC, hlen - j0);
    __syncthreads();
    float hmax = 0.f;
    for (int f = tid; f < jn * (D / 4); f += THREADS) {
      const int jj = f / (D / 4), q4 = f % (D / 4);
      const int64_t item = indices[hbeg + j0 + jj];
      float4 v;
      if (!REGION || q4 < DH / 4)
        v = reinterpret_cast<const float4*>(p.eh + item * p.item_dim)[q4];
      else
        v = reinterpret_cast<const float4*>(p.er + region_of[item] * p.region_dim)[q4 - DH / 4];
      reinterpret_cast<float4*>(hrows)[f] = v;
      hmax = fmaxf(hmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (int jj = tid; jj < jn; jj += THREADS) {
      const int64_t item = indices[hbeg + j0 + jj];
      hid[jj] = (int32_t)item;
      if (DIST && coords) {
        hco[2 * jj] = coords[2 * item];
        hco[2 * jj + 1] = coords[2 * item + 1];
      }
    }
    const float mh = block_max(hmax, red);   // contains the barrier that publishes the chunk
    const float Snew = pow2_scale(tmax * mh);
    const float ratio = Snew / St;           // exact: both powers of two
#pragma unroll
    for (int k = 0; k < DH; ++k) tv[k] *= ratio;
    St = Snew;
    const float invS = 1.f / (Sw * St);
    epi.rescale(Eimg, hh, Sw * St, invS);
    const float invSt = 1.f / St;

    for (int jj = 0; jj < jn; ++jj) {
      const float* hr = hrows + jj * D + hh * DH;
      floatx16 acc[HB];
#pragma unroll
      for (int hb = 0; hb < HB; ++hb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[hb][r] = epi.init(hb * 16 + r);
      float sd = 0.f;
      uint4 an[HB][NPC];
      if constexpr (PREF) {
#pragma unroll
        for (int hb = 0; hb < HB; ++hb)
#pragma unroll
          for (int q = 0; q < NPC; ++q) an[hb][q] = A16[((hb * KS) * NPC + q) * 64 + lane];
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        uint4 ac[HB][NPC];
#pragma unroll
        for (int hb = 0; hb < HB; ++hb)
#pragma unroll
          for (int q = 0; q < NPC; ++q)
            ac[hb][q] = PREF ? an[hb][q] : A16[((hb * KS + s) * NPC + q) * 64 + lane];
        if (PREF && s + 1 < KS) {
#pragma unroll
          for (int hb = 0; hb < HB; ++hb)
#pragma unroll
            for (int q = 0; q < NPC; ++q) an[hb][q] = A16[((hb * KS + s + 1) * NPC + q) * 64 + lane];
        }
        const float4 h0 = *reinterpret_cast<const float4*>(hr + 8 * s);
        const float4 h1 = *reinterpret_cast<const float4*>(hr + 8 * s + 4);
        float x[8];
        x[0] = tv[8 * s + 0] * h0.x;
        x[1] = tv[8 * s + 1] * h0.y;
        x[2] = tv[8 * s + 2] * h0.z;
        x[3] = tv[8 * s + 3] * h0.w;
        x[4] = tv[8 * s + 4] * h1.x;
        x[5] = tv[8 * s + 5] * h1.y;
        x[6] = tv[8 * s + 6] * h1.z;
        x[7] = tv[8 * s + 7] * h1.w;
#pragma unroll
        for (int e = 0; e < 8; ++e) sd += x[e];
        half8 xp[NPC];
        split_pieces<NPC>(x, xp);
#pragma unroll
        for (int hb = 0; hb < HB; ++hb) {
          half8 ap_[NPC];
#pragma unroll
          for (int q = 0; q < NPC; ++q) ap_[q] = *reinterpret_cast<const half8*>(&ac[hb][q]);
          acc[hb] = mfma_pieces<NPC>(ap_, xp, acc[hb]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (DIST) {
        float ll0, ll1;
        if (coords) {
          ll0 = (float)fabs(clat - hco[2 * jj]);
          ll1 = (float)fabs(clon - hco[2 * jj + 1]);
        } else {
          ll0 = (float)llrow[2 * (int64_t)hid[jj]];
          ll1 = (float)llrow[2 * (int64_t)hid[jj] + 1];
        }
        const float fs = dist_feature(dw, ll0, ll1) * St;   // exact power-of-two scaling
#pragma unroll
        for (int hb = 0; hb < HB; ++hb) acc[hb] = mfma32(Adist[hb * 64 + lane], fs, acc[hb]);
      }
      float ap = 0.f;
#pragma unroll
      for (int hb = 0; hb < HB; ++hb)
#pragma unroll
        for (int r = 0; r < 16; ++r) ap += epi.term(hb * 16 + r, acc[hb][r], invS);
      const float a = ap + __shfl_xor(ap, 32);
      const float sv = (sd + __shfl_xor(sd, 32)) * invSt;
      const bool keep = hid[jj] != (int32_t)c;
      const float e = expf(a) * (keep ? 1.f : 0.f);
      if (tab.e) {   // pair-table mode: the pair's two terms instead of the user's sums
        if (valid && hh == 0) {
          tab_put(tab, hbeg + j0 + jj, c - tab.col0, e, e * sv);
        }
        continue;
      }
      in_hist |= !keep;
      S += e;
      N += e * sv;
    }
  }
  if (tab.e) return;

  const float logit = finish_logit(S, N, p.beta, hlen == 0);
  const bool isnan_ = logit != logit;
  float sc = sigmoidf_ref(logit);
  if (isnan_) sc = __builtin_nanf("");
  if (in_hist) sc = -1.f;
  if (valid && hh == 0) scores[(int64_t)cat_user_slot() * score_ld + c] = sc;
  if (nan_count) {
    const unsigned long long m = __ballot(valid && hh == 0 && !in_hist && isnan_);
    if (lane == 0 && m) atomicAdd(nan_count, (int32_t)__popcll(m));
  }
}

// ---------------------------------------------------------------------------------------------
// Split-fp16 catalog scorer, item-side factorisation ("x3b"):
//   W1 (h_j (.) t_c) = (W1 diag(h_j)) t_c = A_j t_c
// A_j (H x D) is formed ONCE per history item per workgroup, in fp32 (a_ik = w_ik * h_jk), then
// scaled by S_A and split into fp16 hi/lo in MFMA-A fragment order in an LDS ring (all 512
// threads build it, one barrier per group of items); t_c is scaled by S_t and split ONCE per
// candidate into B fragments that stay in VGPRs for the whole sweep. The per-(c, j) VALU work
// is then only the epilogue and h_j . t_c -- no per-pair conversions.
// ---------------------------------------------------------------------------------------------
template <int DH, int HB, bool DIST, int NW = WAVES, int NPC = 2>
struct CfgB {
  static constexpr int D = 2 * DH;
  static constexpr int KS = DH / 8;
  static constexpr int NE = HB * KS * 64;             // uint4 fragment entries per item and piece
  static constexpr int IB = NE * 16 * NPC;            // bytes per item (all pieces)
  static constexpr int G = IB <= 16384 ? 4 : (IB <= 32768 ? 2 : 1);   // items per ring group
  // LDS chunk rows; fp16x6 keeps 32 (the s tile below) even where 64 would fit (64-row chunks
  // without the s tile: -1..-3 %, profiles/r2/jcb_ab)
  static constexpr int JCB = (NPC == 3) ? 32 : (2 * G * IB + 64 * D * 4 > 140 * 1024 ? 32 : 64);
  static constexpr int EPT = (NE + NW * 64 - 1) / (NW * 64);  // build entries per thread
  static constexpr int ADIST = DIST ? HB * 64 : 0;
  static constexpr int EPI = 2 * 2 * HB * 16;
  // PIPE: the epilogue of item j-1 interleaved with item j's MFMAs (two accumulator sets, b1 / w2
  // in VGPRs) -- fits 256 VGPRs for D, H <= 64. Wider: one accumulator set, epilogue right after
  // the item's MFMAs (the SIMD's other wave overlaps it), b1 / w2 read from LDS (Epi16<HB, false>).
  // fp16x6 (NPC = 3) pipelines too, with b1 / w2 read from LDS (EREGS = false) to stay within
  // 256 VGPRs; without the pipeline the per-group barrier lines up both waves of a SIMD, so their
  // MFMA and VALU phases coincide instead of overlapping
  static constexpr bool PIPE = HB <= 2 && DH <= 32;
  static constexpr bool EREGS = PIPE && NPC == 2;   // b1 / w2 pre-scaled in VGPRs
  // fp16x6 pipeline: one candidate scale S_t per WAVE (not per lane), so S = S_A * S_t is
  // wave-uniform and each wave keeps S*b1 and w2/S in its own LDS slot (Epi16L): acc starts at
  // S*b1 and the epilogue is relu + fma (3 VALU per value instead of 4), no VGPRs spent
  static constexpr bool WLDS = PIPE && !EREGS;
  static constexpr int ESCL = WLDS ? NW * EPI : 0;
  static constexpr size_t REST = size_t(ADIST) * 4 + size_t(EPI) * 4 + size_t(ESCL) * 4 + 64 +
                                 size_t(JCB) * D * 4 + size_t(JCB) * 4 + (DIST ? size_t(JCB) * 16 : 0);
  static constexpr size_t BYTES = size_t(2) * G * IB + REST;
  static_assert(!PIPE || G % 2 == 0, "the pipelined steps alternate two accumulator sets per item");
};

// NW = waves per workgroup (2 per SIMD at 8). D, H <= 64 pipeline the epilogue (CfgB::PIPE).
template <int DH, int HB, int VAR, int NW, int NPC>
__global__ void __launch_bounds__(NW * 64, NW >= 8 ? 1 : 8 / NW)   // >= 2 waves per SIMD per CU
catalog_score_x3b_kernel(DevParams p, const int64_t* __restrict__ indptr,
                         const int64_t* __restrict__ indices, const int32_t* __restrict__ users,
                         const int64_t* __restrict__ region_of, const double* __restrict__ coords,
                         const double* __restrict__ latlon_mat, float* __restrict__ scores,
                         int64_t score_ld, int32_t* __restrict__ nan_count, TableOut tab) {
  constexpr bool REGION = VarT<VAR>::REGION;
  constexpr bool DIST = VarT<VAR>::DIST;
  using C = CfgB<DH, HB, DIST, NW, NPC>;
  constexpr int D = C::D, KS = C::KS, NE = C::NE, G = C::G, JCB = C::JCB, EPT = C::EPT;
  constexpr int THREADS = NW * 64, CAND_PER_BLOCK = NW * 32;   // shadow the 8-wave defaults
  constexpr bool PIPE = C::PIPE;
  // s = h_j . t_c for the chunk's 32 items on the matrix pipe (one 32x32 tile per wave and chunk,
  // the same split-fp16 3-product scheme) instead of a 2*DH-term VALU dot per item and lane
  constexpr bool SMF = JCB == 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);       // [2 groups][G items][piece][NE]
  float* Adist = reinterpret_cast<float*>(ring + 2 * G * NPC * NE);
  float* Eimg = Adist + C::ADIST;
  float* Escl = Eimg + C::EPI;          // WLDS: per wave [S*b1 | w2/S] (EPI floats each)
  float* red = Escl + C::ESCL;
  float* hrows = red + 16;
  int32_t* hid = reinterpret_cast<int32_t*>(hrows + JCB * D);
  double* hco = reinterpret_cast<double*>(hid + JCB);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
  int64_t hbeg, hlen;
  if (tab.e) {   // pair-table mode: a group of tab.gi rows of the item list
    hbeg = (int64_t)cat_user_slot() * tab.gi;
    hlen = std::min<int64_t>(tab.gi, tab.nitems - hbeg);
  } else {
    const int64_t u = users[cat_user_slot()];
    hbeg = indptr[u];
    hlen = indptr[u + 1] - hbeg;
  }
  const int64_t c = tab.col0 + (int64_t)cat_tile() * CAND_PER_BLOCK + wave * 32 + (lane & 31);
  const bool valid = c < p.P && (!tab.e || c < tab.col0 + tab.cols);
  const int64_t cc = valid ? c : p.P - 1;

  // ---- this thread's W1 values for the fragment entries it builds (fp32, unscaled)
  float wv[EPT][8];
  float wmax = 0.f;
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * THREADS;
    const int ln = e & 63, s = (e >> 6) % KS, hb = (e >> 6) / KS;
    const int i = hb * 32 + (ln & 31), k0 = (ln >> 5) * DH + 8 * s;
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      wv[q][x] = (e < NE && i < p.H) ? p.w1[(int64_t)i * p.din + k0 + x] : 0.f;
      wmax = fmaxf(wmax, fabsf(wv[q][x]));
    }
  }
  const float Wmax = block_max_n<NW>(wmax, red);
  if (DIST) {
    for (int f = tid; f < C::ADIST; f += THREADS) {
      const int ln = f & 63, hb = f >> 6, i = hb * 32 + (ln & 31);
      Adist[f] = (i < p.H) ? p.w1[(int64_t)i * p.din + D + (ln >> 5)] : 0.f;
    }
  }
  for (int f = tid; f < C::EPI; f += THREADS) {
    const int which = f / (2 * HB * 16), rem = f % (2 * HB * 16);
    const int hh2 = rem / (HB * 16), hr = rem % (HB * 16), hb = hr / 16, r = hr % 16;
    const int i = acc_row(hb, r, hh2);
    Eimg[f] = (i < p.H) ? (which == 0 ? p.b1[i] : p.w2[i]) : 0.f;
  }

  // ---- candidate operand: t_c scaled by S_t (fp32 copy for h . t) and its fp16 hi/lo B fragments
  float tv[DH];
  {
    const float* src = (REGION && hh) ? p.er + region_of[cc] * p.region_dim
                                      : p.et + cc * p.item_dim + (REGION ? 0 : hh * DH);
#pragma unroll
    for (int q = 0; q < DH / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(src)[q];
      tv[4 * q] = v.x;
      tv[4 * q + 1] = v.y;
      tv[4 * q + 2] = v.z;
      tv[4 * q + 3] = v.w;
    }
  }
  float tmax = 0.f;
#pragma unroll
  for (int k = 0; k < DH; ++k) tmax = fmaxf(tmax, fabsf(tv[k]));
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
  if constexpr (C::WLDS) {   // one scale for the wave's 32 candidates (its pieces reach 2^-39 of it)
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, o));
  }
  const float St = pow2_scale(tmax);
  const float invSt = 1.f / St;
  half8 tb[KS][NPC];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      tv[8 * s + e] *= St;
      x[e] = tv[8 * s + e];
    }
    split_pieces<NPC>(x, tb[s]);
  }
  double clat = 0.0, clon = 0.0;
  DistW dw{0.f, 0.f, 0.f};
  const double* llrow = nullptr;
  if (DIST) {
    if (coords) {
      clat = coords[2 * cc];
      clon = coords[2 * cc + 1];
    } else {
      llrow = latlon_mat + cc * p.P * 2;
    }
    dw = load_distw<VAR>(p, hh);
  }

  float S = 0.f, N = 0.f;
  bool in_hist = false;
  // b1 / w2 pre-scaled in VGPRs when pipelined; read from LDS (unscaled, one fma per use) when wide
  std::conditional_t<C::WLDS, Epi16L<HB>, Epi16<HB, C::EREGS>> epi;

  // build the fragments of chunk-local item jj into ring slot (grp, it)
  // build the fragments of chunk-local item jj into ring slot (grp, it); wv is pre-scaled by S_A
  auto build = [&](int jj, int grp, int it) {
    const float* hr = hrows + jj * D;
    uint4* dst = ring + ((grp * G + it) * NPC) * NE;
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * THREADS;
      if (e < NE) {
        const int ln = e & 63, s = (e >> 6) % KS;
        const int k0 = (ln >> 5) * DH + 8 * s;
        const float4 h0 = *reinterpret_cast<const float4*>(hr + k0);
        const float4 h1 = *reinterpret_cast<const float4*>(hr + k0 + 4);
        float a[8];
        a[0] = wv[q][0] * h0.x;
        a[1] = wv[q][1] * h0.y;
        a[2] = wv[q][2] * h0.z;
        a[3] = wv[q][3] * h0.w;
        a[4] = wv[q][4] * h1.x;
        a[5] = wv[q][5] * h1.y;
        a[6] = wv[q][6] * h1.z;
        a[7] = wv[q][7] * h1.w;
        half8 pc[NPC];
        split_pieces<NPC>(a, pc);
#pragma unroll
        for (int q2 = 0; q2 < NPC; ++q2) dst[q2 * NE + e] = *reinterpret_cast<const uint4*>(&pc[q2]);
      }
    }
  };

  float Sacc = 1.f, invS = 1.f;
  int64_t j0 = 0;   // history chunk base (the step's table-mode write needs it)
  floatx16 sacc;                 // SMF: s tile [32 chunk items x 32 candidates], scaled by Sh*St
  float invShSt = 1.f;

  // One pipeline step: the MFMA chain of item `cur` (A_j from the ring slot `src`, t_c from VGPRs)
  // into accN, with the VALU epilogue of the previous item (accP, chunk-local `prev`) cut into KS
  // slices placed between the K-steps, so the matrix pipe and the VALU work side by side inside
  // one wave (A/B: profiles/r1/ab_*.json). `live` = false makes the epilogue a no-op (its result
  // is selected away), keeping the control flow uniform inside the step.
  // the pair's e and e*s from its attention logit partial ap (and, without SMF, the h.t partial
  // sd): table-mode stores or the user's running sums
  auto tail = [&](int pj, float ap, float sd, bool live) {
    const float2 aph = lane_halves(ap);
    const float a = aph.x + aph.y;
    float sv;
    if (SMF) {   // item pj's row of the s tile: register ((pj/8)*4 + pj%4) of lane half (pj/4)%2
      const float2 sh2 = lane_halves(sacc[((pj >> 3) << 2) | (pj & 3)]);
      sv = (((pj >> 2) & 1) ? sh2.y : sh2.x) * invShSt;
    } else {
      const float2 sdh = lane_halves(sd);
      sv = (sdh.x + sdh.y) * invSt;
    }
    const bool keep = hid[pj] != (int32_t)c;
    const float e = expf(a) * (keep ? 1.f : 0.f);
    if (live) {
      if (tab.e) {
        if (valid && hh == 0) {
          tab_put(tab, hbeg + j0 + pj, c - tab.col0, e, e * sv);
        }
      } else {
        in_hist |= !keep;
        S += e;
        N += e * sv;
      }
    }
    };

  auto step = [&](auto do_mma, auto do_epi, const uint4* src, floatx16 (&accN)[HB],
                  const floatx16 (&accP)[HB], int cur, int prev, bool live) {
    constexpr bool MMA = decltype(do_mma)::value;
    constexpr bool EPIL = decltype(do_epi)::value;
    constexpr int NV = HB * 16;                 // accumulator values per lane
    constexpr int VPS = (NV + KS - 1) / KS;     // epilogue values per K-step slice
    constexpr int QPS = (DH / 4 + KS - 1) / KS; // h . t float4 groups per slice
    const int pj = live ? prev : 0;
    const float* hr = hrows + pj * D + hh * DH;
    float sd = 0.f, ap = 0.f;
    if (MMA) {
#pragma unroll
      for (int hb = 0; hb < HB; ++hb)
#pragma unroll
        for (int r = 0; r < 16; ++r) accN[hb][r] = epi.init(hb * 16 + r);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (MMA) {
#pragma unroll
        for (int hb = 0; hb < HB; ++hb) {
          half8 ap_[NPC];
#pragma unroll
          for (int q = 0; q < NPC; ++q) {
            const uint4 u4 = src[q * NE + (hb * KS + s) * 64 + lane];
            ap_[q] = *reinterpret_cast<const half8*>(&u4);
          }
          accN[hb] = mfma_pieces<NPC>(ap_, tb[s], accN[hb]);
        }
      }
      if constexpr (EPIL) {
#pragma unroll
        for (int v = s * VPS; v < (s + 1) * VPS && v < NV; ++v)
          ap += epi.term(v, accP[v / 16][v % 16], invS);
      }
      if (EPIL && !SMF) {
#pragma unroll
        for (int q = s * QPS; q < (s + 1) * QPS && q < DH / 4; ++q) {
          const float4 hv = *reinterpret_cast<const float4*>(hr + 4 * q);
          sd = __builtin_fmaf(tv[4 * q], hv.x, sd);
          sd = __builtin_fmaf(tv[4 * q + 1], hv.y, sd);
          sd = __builtin_fmaf(tv[4 * q + 2], hv.z, sd);
          sd = __builtin_fmaf(tv[4 * q + 3], hv.w, sd);
        }
      }
    }
    if (DIST && MMA) {   // the 2 distance columns of item `cur`: exact fp32 MFMA K-step
      float ll0, ll1;
      if (coords) {
        ll0 = (float)fabs(clat - hco[2 * cur]);
        ll1 = (float)fabs(clon - hco[2 * cur + 1]);
      } else {
        ll0 = (float)llrow[2 * (int64_t)hid[cur]];
        ll1 = (float)llrow[2 * (int64_t)hid[cur] + 1];
      }
      const float fs = dist_feature(dw, ll0, ll1) * Sacc;   // exact power-of-two scaling
#pragma unroll
      for (int hb = 0; hb < HB; ++hb) accN[hb] = mfma32(Adist[hb * 64 + lane], fs, accN[hb]);
    }
    if constexpr (EPIL) tail(pj, ap, sd, live);
  };

  // wide shapes (no PIPE): item `cur`'s MFMAs in passes of two 32-unit hidden blocks, each pass's
  // epilogue right after it (one pass of accumulators live), then the pair's tail
  auto step_wide = [&](const uint4* src, int cur) {
    constexpr int HS = HB < 2 ? HB : 2;
    float ap = 0.f;
#pragma unroll 1
    for (int h0 = 0; h0 < HB; h0 += HS) {
      floatx16 acc[HS];
#pragma unroll
      for (int hb = 0; hb < HS; ++hb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[hb][r] = epi.init((h0 + hb) * 16 + r);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int hb = 0; hb < HS; ++hb) {
          half8 ap_[NPC];
#pragma unroll
          for (int q = 0; q < NPC; ++q) {
            const uint4 u4 = src[q * NE + ((h0 + hb) * KS + s) * 64 + lane];
            ap_[q] = *reinterpret_cast<const half8*>(&u4);
          }
          acc[hb] = mfma_pieces<NPC>(ap_, tb[s], acc[hb]);
        }
      }
#pragma unroll
      for (int hb = 0; hb < HS; ++hb)
#pragma unroll
        for (int r = 0; r < 16; ++r) ap += epi.term((h0 + hb) * 16 + r, acc[hb][r], invS);
    }
    float sd = 0.f;   // without the s tile (JCB = 64): h_j . t_c as a VALU dot on this lane half
    if constexpr (!SMF) {
      const float* hr = hrows + cur * D + hh * DH;
#pragma unroll
      for (int q = 0; q < DH / 4; ++q) {
        const float4 hv = *reinterpret_cast<const float4*>(hr + 4 * q);
        sd = __builtin_fmaf(tv[4 * q], hv.x, sd);
        sd = __builtin_fmaf(tv[4 * q + 1], hv.y, sd);
        sd = __builtin_fmaf(tv[4 * q + 2], hv.z, sd);
        sd = __builtin_fmaf(tv[4 * q + 3], hv.w, sd);
      }
    }
    tail(cur, ap, sd, true);
  };

  float SAcur = 1.f;
  floatx16 acc2[2][HB];   // PIPE: the accumulators of even / odd chunk-local items
  for (j0 = 0; j0 < hlen; j0 += JCB) {
    const int jn = (int)std::min<int64_t>(JCB, hlen - j0);
    __syncthreads();
    float hmax = 0.f;
    for (int f = tid; f < jn * (D / 4); f += THREADS) {
      const int jj = f / (D / 4), q4 = f % (D / 4);
      const int64_t item = indices[hbeg + j0 + jj];
      float4 v;
      if (!REGION || q4 < DH / 4)
        v = reinterpret_cast<const float4*>(p.eh + item * p.item_dim)[q4];
      else
        v = reinterpret_cast<const float4*>(p.er + region_of[item] * p.region_dim)[q4 - DH / 4];
      reinterpret_cast<float4*>(hrows)[f] = v;
      hmax = fmaxf(hmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (int jj = tid; jj < jn; jj += THREADS) {
      const int64_t item = indices[hbeg + j0 + jj];
      hid[jj] = (int32_t)item;
      if (DIST && coords) {
        hco[2 * jj] = coords[2 * item];
        hco[2 * jj + 1] = coords[2 * item + 1];
      }
    }
    const float Hm = block_max_n<NW>(hmax, red);                        // barrier: chunk published
    const float SA = pow2_scale(Wmax * Hm);
    const float rs = SA / SAcur;                                  // exact power-of-two ratio
    if (SMF) {
      const float Sh = pow2_scale(Hm);
      invShSt = 1.f / (Sh * St);
      const int m = lane & 31;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        float x[8];
        const float* hp = hrows + m * D + hh * DH + 8 * s;
        const float4 h0 = *reinterpret_cast<const float4*>(hp);
        const float4 h1 = *reinterpret_cast<const float4*>(hp + 4);
        const bool ok = m < jn;
        x[0] = ok ? h0.x * Sh : 0.f; x[1] = ok ? h0.y * Sh : 0.f;
        x[2] = ok ? h0.z * Sh : 0.f; x[3] = ok ? h0.w * Sh : 0.f;
        x[4] = ok ? h1.x * Sh : 0.f; x[5] = ok ? h1.y * Sh : 0.f;
        x[6] = ok ? h1.z * Sh : 0.f; x[7] = ok ? h1.w * Sh : 0.f;
        half8 hpc[NPC];
        split_pieces<NPC>(x, hpc);
        sacc = mfma_pieces<NPC>(hpc, tb[s], sacc);
      }
    }
#pragma unroll
    for (int q = 0; q < EPT; ++q)
#pragma unroll
      for (int x = 0; x < 8; ++x) wv[q][x] *= rs;
    SAcur = SA;
    Sacc = SA * St;
    invS = 1.f / Sacc;
    if constexpr (C::WLDS) {   // this wave's S*b1 and w2/S (S is wave-uniform); the barrier
      float* mine = Escl + wave * C::EPI;   // after the first builds publishes them
      for (int f = lane; f < C::EPI; f += 64) mine[f] = Eimg[f] * (f < 2 * HB * 16 ? Sacc : invS);
      epi.rescale(mine, hh, Sacc, invS);
    } else {
      epi.rescale(Eimg, hh, Sacc, invS);
    }
    const int ngroups = (jn + G - 1) / G;
#pragma unroll
    for (int it = 0; it < G; ++it)
      if (it < jn) build(it, 0, it);
    __syncthreads();
    int prev = -1;                      // chunk-local item whose epilogue is pending in accP
    for (int g = 0; g < ngroups; ++g) {
      if (g + 1 < ngroups) {
#pragma unroll
        for (int it = 0; it < G; ++it) {
          const int jj = (g + 1) * G + it;
          if (jj < jn) build(jj, (g + 1) & 1, it);
        }
      }
#pragma unroll
      for (int it = 0; it < G; ++it) {
        const int jj = g * G + it;
        if (jj < jn) {
          const uint4* src = ring + (((g & 1) * G + it) * NPC) * NE;
          if constexpr (PIPE) {   // item jj into acc2[jj & 1] (G even: static), item jj - 1 from the other
            step(std::true_type{}, std::true_type{}, src, acc2[it & 1], acc2[(it + 1) & 1], jj, prev,
                 prev >= 0);
            prev = jj;
          } else {
            step_wide(src, jj);
          }
        }
      }
      __syncthreads();
    }
    if (PIPE && prev >= 0) {   // drain: epilogue of the chunk's last item, no MFMAs
      if (prev & 1)
        step(std::false_type{}, std::true_type{}, ring, acc2[0], acc2[1], 0, prev, true);
      else
        step(std::false_type{}, std::true_type{}, ring, acc2[1], acc2[0], 0, prev, true);
    }
  }
  if (tab.e) return;

  const float logit = finish_logit(S, N, p.beta, hlen == 0);
  const bool isnan_ = logit != logit;
  float sc = sigmoidf_ref(logit);
  if (isnan_) sc = __builtin_nanf("");
  if (in_hist) sc = -1.f;
  if (valid && hh == 0) scores[(int64_t)cat_user_slot() * score_ld + c] = sc;
  if (nan_count) {
    const unsigned long long m = __ballot(valid && hh == 0 && !in_hist && isnan_);
    if (lane == 0 && m) atomicAdd(nan_count, (int32_t)__popcll(m));
  }
}

// ---------------------------------------------------------------------------------------------
// The fp16x6 item-side kernel on v_mfma_f32_16x16x32_f16 ("x6n", D in {32, 64, 128}, H <= 256 in
// hidden-unit slices, every variant: basic, region, region_distance, distance): the x3b
// factorisation A_j t_c, the same six products of exact hi / mid / lo f16 pieces, the same per-wave
// candidate scale and pipelined epilogue, in 16 x 16 output tiles:
//   A (16 hidden x 32 dims)    lane l: hidden 16 m + (l & 15), dims 32 s + 8 (l >> 4) .. + 8 (LDS ring)
//   B (32 dims x 16 cands)     lane l: candidate 16 nb + (l & 15), the same dims (VGPRs, 2 blocks nb)
//   C (16 hidden x 16 cands)   lane l: candidate (l & 15), hidden 16 m + 4 (l >> 4) + r
// Each A fragment feeds the wave's two candidate blocks. A 16x16x32 MFMA takes half the cycles of
// a 32x32x16 one for half the work, so the same 1,536 matrix cycles per item and wave; what the
// shape changes is the clock the chip holds under the load (MI355X_MICROARCH.md, DVFS give-back
// item 7) and the issue pressure (an MFMA holds the SIMD's vector issue 8 of its 16 cycles instead
// of 8 of 32). The attention logit of a candidate is summed over the four lane groups by one
// v_permlane32_swap + one v_permlane16_swap for both candidate blocks at once; s = h_j . t_c comes
// from a per-chunk s tile (items x candidates) that each wave parks in its own LDS slot in
// [candidate][item] order, one ds_read per pair. The distance variants' two extra inputs
// sigmoid(dist_layer(scale * |dlat, dlng|)) (model.py:265-267, 369-371) are exact fp32 MFMA
// K-steps: per pair of 16-hidden blocks, two v_mfma_f32_16x16x1_4b_f32 (one per feature) whose four
// blocks are the pair's four 16 x 16 tiles (hidden block, candidate block); A = the W1 distance
// column of the block's hidden units, B = the pair's feature scaled by S. Each lane computes ONE
// feature of one pair -- lane group g: feature g >> 1 of candidate block g & 1 -- and one
// v_permlane32_swap hands every lane both features of its block.
// ---------------------------------------------------------------------------------------------
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx4 mfma16n(half8 a, half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// the six fp16x6 products, smallest terms first (as mfma_pieces<3>)
__device__ __forceinline__ floatx4 mfma16n_pieces(const half8 (&a)[3], const half8 (&b)[3], floatx4 c) {
  c = mfma16n(a[2], b[0], c);
  c = mfma16n(a[1], b[1], c);
  c = mfma16n(a[0], b[2], c);
  c = mfma16n(a[1], b[0], c);
  c = mfma16n(a[0], b[1], c);
  c = mfma16n(a[0], b[0], c);
  return c;
}

// A "unit" is one item's A_j restricted to MB blocks of 16 hidden units; NHU units make the item,
// whose logit partials are summed before the tail. The ring holds 2 groups of GU units: GU = 2
// where a unit is <= 24 KiB, else 1 (a whole D = H = 128 item, 96 KiB, does not fit twice in the
// 160 KiB LDS, hence units).
// compile-time hidden slices of one x6n step: the unit it multiplies, the unit it finishes and the
// unit it builds
template <int C, int P, int B>
struct X6Slices {
  static constexpr int cur = C, prev = P, built = B;
};

// The distance features are formed one item ahead, at MFMA group 1 of the item before (region_distance
// table block, same process, start of the item's own step / group 1 / 4 / 7: D = H = 64 2.282 /
// 2.251 / 2.289 / 2.250 ms, D = H = 128 8.002 / 7.852 / 7.966 / 7.926 ms -- profiles/r5/feats_at).
// The distance term as 16 VALU FMAs per 16-hidden block on the accumulators' initial values
// (acc = S b1 + wd0 f0 + wd1 f1) instead of the f32 MFMA K-step: 2.256 vs 2.246 ms (D = 64), 8.017
// vs 8.058 ms (D = 128) -- a wash, not kept (profiles/r5/dist_valu).
// With the cheaper feature (v_exp / v_rcp, the folded exponent) group 3 wins at D = 64: table block
// 2.093 / 2.075 / 2.077 ms and the config-4 job 0.616 / 0.614 / 0.612 s at groups 1 / 0 / 3
// (profiles/r5/fa); D = 128 keeps group 1 (unmeasured since).
constexpr int X6N_FEATS_AT = -1;   // -1: 3 at D <= 64, 1 at D = 128
// The distance term as two v_mfma_f32_16x16x1_4b_f32 per PAIR of 16-hidden blocks (the four 16x16
// tiles (m, nb) of the pair as the instruction's four blocks, K = 1 feature each; layout probed,
// scripts/probes/mfma_4b_layout.hip, profiles/r5/d4b) instead of two v_mfma_f32_16x16x4_f32 per
// block with half their K unused: region_distance table block 2.278 -> 2.251 ms (D = H = 64),
// 8.193 -> 7.865 ms (D = H = 128), same process. (Dropping the latlon_mat branch of the feature
// computation as well: 2.208 / 8.140 ms -- mixed; the config-4 region_distance job without it
// 0.631 / 0.637 s against 0.640 / 0.636 s interleaved, profiles/r5/llm -- not pursued.)
__device__ __forceinline__ floatx16 mfma4b(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c, 0, 0, 0);
}
// Tried and not kept (profiles/r5/prio_split, standalone table blocks, same process): static
// priority 1 for waves 4-7 (MI355X_MICROARCH.md, two waves per SIMD, item 4) 2.026 -> 2.014 ms at
// D = H = 64, 7.474 -> 7.479 ms at D = H = 128; the D = 128 build's two entries at a quarter and
// three quarters of the step instead of both at its middle 7.474 -> 7.509 ms. Packed fp32 VALU
// (v_pk_fma_f32 for the two candidate blocks' epilogue chains, v_pk_mul_f32 in the build: 498 ->
// 437 VALU per 4-item block at D = 64) 1.983 -> 1.998 ms at D = H = 64, 7.198 -> 7.228 ms at 128
// (profiles/r5/pk): the block is not issue-bound.

// (the A/B switches of the round-5 x6n work are constants since round 6: EPI_PREFETCH and EPI_REGS
// are described, with their measurements, where they are used below)
constexpr bool X6N_EPI_PREFETCH = true;
constexpr bool X6N_EPI_REGS = true;
constexpr int X6N_W1_VGPRS = 32;   // W1 values a thread may hold in VGPRs (more: W1G). 16 (W1 from L2
                                   // at D = H = 128 too): 20 -> 23 spilled VGPRs there, so not that
template <int D, int MB, int NHU, bool DIST = false>
struct CfgN {
  static constexpr int KS = D / 32;                    // K-steps of 32 dims
  static constexpr int NE = MB * KS * 64;              // uint4 entries per unit and piece
  static constexpr int IB = NE * 16 * 3;               // LDS bytes per unit (three pieces)
  static constexpr int GU = IB <= 24576 ? 2 : 1;       // units per ring group
  static constexpr int NW = 8, THREADS = NW * 64, CPB = NW * 32;
  static constexpr int EPT = (NE + THREADS - 1) / THREADS;   // build entries per thread and unit
  static constexpr int HPU = MB * 16;                  // hidden units per unit
  static constexpr int HP = HPU * NHU;                 // hidden units, padded
  static constexpr int EPI = 2 * HP;                   // [b1 | w2] by hidden unit
  // distance columns of W1: [hidden][4] (2, 3 zero) for the f32 MFMA K-step
  static constexpr int ADN = DIST ? HP * 4 : 0;
  static constexpr size_t bytes(int jcb) {
    return size_t(2) * GU * IB + size_t(EPI) * 4 + size_t(NW) * EPI * 4 + 64 + size_t(jcb) * D * 4 +
           size_t(jcb) * 4 + size_t(NW) * 32 * (jcb + 1) * 4 + size_t(ADN) * 4 + (DIST ? size_t(jcb) * 16 : 0);
  }
  // chunk rows (the s tile's items): 32, or 16 where 32 does not fit the LDS (D = 128 with 256
  // hidden units: the per-wave [S b1 | w2 / S] copies grow with H)
  static constexpr int JCB = bytes(32) <= 160 * 1024 ? 32 : 16;
  static constexpr int SVP = JCB + 1;                  // s image pitch (floats): [cand][item]
  static constexpr size_t BYTES = bytes(JCB);
  // groups per round: a round of GQ groups (GQ * GU units) spans whole items, so every step's
  // hidden slices are compile-time; the two ring slots alternate within it
  static constexpr int GQ = (NHU / GU) > 2 ? NHU / GU : 2;
  // W1 read from global memory (L2) at each build instead of held in VGPRs when a thread's
  // share of it would take more than 32 VGPRs (D = 128 with more than 128 hidden units)
  static constexpr bool W1G = NHU * EPT * 8 > X6N_W1_VGPRS;
  static_assert(BYTES <= 160 * 1024, "x6n: LDS");
  static_assert((GQ * GU) % NHU == 0 && GQ % 2 == 0 && GQ <= 4, "x6n: a round of groups spans whole items");
};


template <int D, int MB, int NHU, int VAR>
__global__ void __launch_bounds__(512, 1)
catalog_score_x6n_kernel(DevParams p, const int64_t* __restrict__ indptr,
                         const int64_t* __restrict__ indices, const int32_t* __restrict__ users,
                         const int64_t* __restrict__ region_of, const double* __restrict__ coords,
                         const double* __restrict__ latlon_mat, float* __restrict__ scores,
                         int64_t score_ld, int32_t* __restrict__ nan_count, TableOut tab) {
  constexpr bool REGION = VarT<VAR>::REGION;
  constexpr bool DIST = VarT<VAR>::DIST;
  using C = CfgN<D, MB, NHU, DIST>;
  constexpr int KS = C::KS, NE = C::NE, GU = C::GU, JCB = C::JCB, EPT = C::EPT, HP = C::HP;
  constexpr int HPU = C::HPU, EPI = C::EPI, NW = C::NW, THREADS = C::THREADS, CPB = C::CPB;
  constexpr int SVP = C::SVP;
  constexpr int DH = D / 2;   // region variants: dims [DH, D) come from embed_region
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* ring = reinterpret_cast<uint4*>(smem);                    // [2 groups][GU units][piece][NE]
  float* Eimg = reinterpret_cast<float*>(ring + 2 * GU * 3 * NE);  // [b1 | w2] by hidden unit
  float* Escl = Eimg + EPI;                                        // per wave [S*b1 | w2/S]
  float* red = Escl + NW * EPI;
  float* hrows = red + 16;                                         // [JCB][D]
  int32_t* hid = reinterpret_cast<int32_t*>(hrows + JCB * D);
  float* svt = reinterpret_cast<float*>(hid + JCB);                // per wave [32 cands][SVP]
  float* Adn = svt + NW * 32 * SVP;                                // DIST: W1 distance columns [HP][4]
  double* hco = reinterpret_cast<double*>(Adn + C::ADN);           // DIST: the chunk's coordinates [JCB][2]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, grp = lane >> 4, l16 = lane & 15;
  const int64_t clim = tab.e ? std::min<int64_t>(p.P, tab.col0 + tab.cols) : p.P;

  // ---- this thread's W1 values for its build entries of every unit (fp32, unscaled); with W1G
  // only their maximum (the build reads them from global memory)
  constexpr bool W1G = C::W1G;
  float wv[W1G ? 1 : NHU][EPT][8];
  float wmax = 0.f;
#pragma unroll
  for (int h = 0; h < NHU; ++h)
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * THREADS;
      const int ln = e & 63, s = (e >> 6) % KS, m = (e >> 6) / KS;
      const int i = HPU * h + 16 * m + (ln & 15), k0 = 32 * s + 8 * (ln >> 4);
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const float w = (e < NE && i < p.H) ? p.w1[(int64_t)i * p.din + k0 + x] : 0.f;
        if constexpr (!W1G) wv[h][q][x] = w;
        wmax = fmaxf(wmax, fabsf(w));
      }
    }
  for (int f = tid; f < EPI; f += THREADS) {
    const int i = f % HP;
    Eimg[f] = (i < p.H) ? (f < HP ? p.b1[i] : p.w2[i]) : 0.f;
  }
  if constexpr (DIST) {
    for (int f = tid; f < C::ADN; f += THREADS) {
      const int i = f >> 2, k = f & 3;
      Adn[f] = (i < p.H && k < 2) ? p.w1[(int64_t)i * p.din + D + k] : 0.f;
    }
  }
  const float Wmax = block_max_n<NW>(wmax, red);   // its barriers also publish Eimg / Adn
  // DIST: this lane's feature row of dist_layer (feature grp & 1, model.py:265 / 369)
  const DistW dw = DIST ? load_distw<VAR>(p, grp >> 1) : DistW{0.f, 0.f, 0.f, 0.f};
  // -log2(e) * (scale * w0, scale * w1, b): the feature's exponent as two FMAs
  const float fk0 = -1.44269504f * (dw.scale * dw.w0), fk1 = -1.44269504f * (dw.scale * dw.w1);
  const float fk2 = -1.44269504f * dw.b;

  float SAcur = 1.f;   // the W1 registers' current scale (rescaled per chunk)

  // Work items: (item group, column tile) in pair-table mode, (user slot, column tile) otherwise.
  // With tab.work (pair-table mode) the workgroup takes items from that counter until they run
  // out -- a work queue, so a shader engine with fewer enabled CUs simply takes fewer (the stream
  // split needs no 32-CU steps); items are tile-major, so a workgroup's candidate operands usually
  // carry over to its next item.
  __shared__ int32_t wi_sh;
  int64_t wslot = cat_user_slot(), wtile = cat_tile(), cur_tile = -1;
  half8 tb[2][KS][3];
  float St = 1.f;
  int64_t cbase = 0, cout = 0;
  bool vout = false;
  double fclat = 0.0, fclon = 0.0;     // DIST: coordinates of this lane's feature candidate
  const double* llrow = nullptr;       // DIST, latlon_mat mode: its row of the matrix
  for (int64_t it = 0;; ++it) {
  if (tab.work) {
    __syncthreads();   // the previous item's readers of wi_sh, hrows, hid and the ring are done
    if (tid == 0) wi_sh = atomicAdd(tab.work, 1);
    __syncthreads();
    const int64_t wi = wi_sh;
    if (wi >= (int64_t)tab.ngroups * tab.ntiles) break;
    wtile = wi / tab.ngroups;
    wslot = wi % tab.ngroups;
  } else if (it > 0) {
    break;
  }
  int64_t hbeg, hlen;
  if (tab.e) {   // pair-table mode: a group of tab.gi rows of the item list
    hbeg = wslot * tab.gi;
    hlen = std::min<int64_t>(tab.gi, tab.nitems - hbeg);
  } else {
    const int64_t u = users[wslot];
    hbeg = indptr[u];
    hlen = indptr[u + 1] - hbeg;
  }
  if (wtile != cur_tile) {   // block-uniform
    cur_tile = wtile;
    cbase = tab.col0 + wtile * CPB + wave * 32;
    // after the lane-group reduction lane L holds candidate cbase + 16 (L >> 5) + (L & 15) (L and
    // L ^ 16 alike): lane groups 0 / 2 carry e, groups 1 / 3 e * s
    cout = cbase + 16 * (lane >> 5) + l16;
    vout = cout < clim;
    if constexpr (DIST) {   // lane group g computes feature g >> 1 of candidate block g & 1
      const int64_t fc = cbase + 16 * (grp & 1) + l16;
      const int64_t fcc = fc < clim ? fc : p.P - 1;
      if (coords) {
        fclat = coords[2 * fcc];
        fclon = coords[2 * fcc + 1];
      } else {
        llrow = latlon_mat + fcc * p.P * 2;
      }
    }
    // ---- candidate operands: two blocks of 16, one scale S_t per wave, split into B fragments
    {
      float tmax = 0.f;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int64_t c = cbase + 16 * nb + l16;
        const int64_t cc = c < clim ? c : p.P - 1;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int k0 = 32 * s + 8 * grp;
          const float* src = (REGION && k0 >= DH) ? p.er + region_of[cc] * p.region_dim + (k0 - DH)
                                                  : p.et + cc * p.item_dim + k0;
          const float4 v0 = reinterpret_cast<const float4*>(src)[0];
          const float4 v1 = reinterpret_cast<const float4*>(src)[1];
          tmax = fmaxf(tmax, fmaxf(fmaxf(fmaxf(fabsf(v0.x), fabsf(v0.y)), fmaxf(fabsf(v0.z), fabsf(v0.w))),
                                   fmaxf(fmaxf(fabsf(v1.x), fabsf(v1.y)), fmaxf(fabsf(v1.z), fabsf(v1.w)))));
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, o));
      St = pow2_scale(tmax);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {   // second read of the rows (L1 / L2 hits): fewer live VGPRs
        const int64_t c = cbase + 16 * nb + l16;
        const int64_t cc = c < clim ? c : p.P - 1;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int k0 = 32 * s + 8 * grp;
          const float* src = (REGION && k0 >= DH) ? p.er + region_of[cc] * p.region_dim + (k0 - DH)
                                                  : p.et + cc * p.item_dim + k0;
          const float4 v0 = reinterpret_cast<const float4*>(src)[0];
          const float4 v1 = reinterpret_cast<const float4*>(src)[1];
          float x[8] = {v0.x * St, v0.y * St, v0.z * St, v0.w * St, v1.x * St, v1.y * St, v1.z * St, v1.w * St};
          split_pieces<3>(x, tb[nb][s]);
        }
      }
    }
  }

  float S = 0.f, N = 0.f;
  bool in_hist = false;
  const float* eb = Escl + wave * EPI;        // S*b1 by hidden unit
  const float* ew = eb + HP;                  // w2/S
  float* sv_mine = svt + wave * 32 * SVP;
  int64_t j0 = 0;
  float pa0 = 0.f, pa1 = 0.f;                 // logit partials of the item's earlier units
  int jn_cur = 1;                             // rows of the current chunk
  float Sd = 1.f;                             // DIST: the accumulators' scale S = S_A * S_t
  float fB0 = 0.f, fB1 = 0.f;                 // DIST: B operands (the item's features, blocks 0 / 1)
  float fN0 = 0.f, fN1 = 0.f;                 // DIST: the next item's, computed one item ahead
  // the distance features of chunk item `item` against this lane's feature candidate, exactly as
  // the other kernels form them (dist_feature: float64 |dlat|, |dlng| cast to float32, x scale,
  // dist_layer row, sigmoid), scaled by S; groups 0 / 1 then hold both blocks' B operands. Formed
  // one item ahead (mid-step of the item before), so its latency (LDS, exp, rcp) hides under
  // that item's MFMAs
  auto feats = [&](int item) __attribute__((always_inline)) {
    item = std::min(item, jn_cur - 1);        // a stale step past the chunk (its MFMAs are unused)
    float ll0, ll1;
    if (coords) {
      ll0 = (float)fabs(fclat - hco[2 * item]);
      ll1 = (float)fabs(fclon - hco[2 * item + 1]);
    } else {
      const int64_t hj = hid[item];
      ll0 = (float)llrow[2 * hj];
      ll1 = (float)llrow[2 * hj + 1];
    }
    // v_exp_f32 + v_rcp_f32 (1 ulp each) instead of the correctly rounded expf and IEEE division
    // (region_distance table block 2.204 -> 2.175 ms, profiles/r5/pk): the feature is an MLP
    // input, so an ulp of it moves the logit far below its own fp32 rounding
    // (the exponent as two FMAs with -log2(e) and the scale folded in: block 2.198 -> 2.183 ms, the
    // config-4 region_distance job 0.631 / 0.629 / 0.631 -> 0.626 / 0.631 / 0.627 s interleaved,
    // profiles/r5/fold); S = Sd is an exact power of two
    const float f = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(ll0, fk0, __builtin_fmaf(ll1, fk1, fk2)))) * Sd;
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(f), __float_as_uint(f), false, false);
    fN0 = __uint_as_float(r[0]);   // every lane: feature 0 / 1 of its candidate block g & 1
    fN1 = __uint_as_float(r[1]);
  };

  // chunk unit u (item u / NHU, hidden slice u % NHU) into ring slot (grp_, it). With NE a multiple
  // of the block size (the D = 64 / 128 shapes) it has no branch, so the scheduler can spread it
  // between the MFMAs of the step it is called from.
  auto build = [&](int u, auto hsc, int grp_, int it) __attribute__((always_inline)) {
    constexpr int HS = decltype(hsc)::value;   // the unit's hidden slice (u % NHU where it matters)
    const float* hr = hrows + (u / NHU) * D;
    uint4* dst = ring + ((grp_ * GU + it) * 3) * NE;
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * THREADS;
      if (NE % THREADS == 0 || e < NE) {
        const int ln = e & 63, s = (e >> 6) % KS;
        const int k0 = 32 * s + 8 * (ln >> 4);
        const float4 h0 = *reinterpret_cast<const float4*>(hr + k0);
        const float4 h1 = *reinterpret_cast<const float4*>(hr + k0 + 4);
        float wg[8];   // W1G: the entry's W1 values scaled by S_A (exact power of two)
        if constexpr (W1G) {
          const int i = HPU * HS + 16 * ((e >> 6) / KS) + (ln & 15);
#pragma unroll
          for (int x = 0; x < 8; ++x) wg[x] = i < p.H ? p.w1[(int64_t)i * p.din + k0 + x] * SAcur : 0.f;
        }
        const float* w = W1G ? wg : wv[W1G ? 0 : HS][q];
        float a[8];
        a[0] = w[0] * h0.x; a[1] = w[1] * h0.y; a[2] = w[2] * h0.z; a[3] = w[3] * h0.w;
        a[4] = w[4] * h1.x; a[5] = w[5] * h1.y; a[6] = w[6] * h1.z; a[7] = w[7] * h1.w;
        half8 pc[3];
        split_pieces<3>(a, pc);
#pragma unroll
        for (int q2 = 0; q2 < 3; ++q2) dst[q2 * NE + e] = *reinterpret_cast<const uint4*>(&pc[q2]);
      }
    }
  };

  // the pair (chunk item pj, this lane's output candidate): the logit partials of the two candidate
  // blocks summed over the lane groups, then e and e * s. No branches: the running sums take
  // selects, and the table rows are written by buffer stores whose offset is out of range (the
  // store dropped) for the lanes that do not write -- so the tail stays in the step's basic block.
  const uint32_t tab_bytes = tab.e ? (uint32_t)(tab.cols * 4) : 0u;
  const int exs = tab.ex ? 2 : 1;   // the es / ex row pitch in units of ld
  auto tail = [&](int pj, float p0, float p1, bool live) __attribute__((always_inline)) {
    const auto r1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(p0), __float_as_uint(p1), false, false);
    const float q = __uint_as_float(r1[0]) + __uint_as_float(r1[1]);   // groups {g, g + 2}
    const auto r2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(q), __float_as_uint(q), false, false);
    const float a = __uint_as_float(r2[0]) + __uint_as_float(r2[1]);   // all four groups
    const float sv = sv_mine[(16 * (lane >> 5) + l16) * SVP + pj];
    const bool keep = hid[pj] != (int32_t)cout;
    const float e = expf(a) * (keep ? 1.f : 0.f);
    in_hist |= live && !keep;
    S += live ? e : 0.f;
    N += live ? e * sv : 0.f;
    const int64_t row = (hbeg + j0 + pj) * tab.ld;
    const int off = (live && vout) ? (int)(cout - tab.col0) * 4 : (int)0x80000000;
    const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(tab.e + row, (short)0, tab_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(tab.es + row * exs, (short)0, tab_bytes * exs, 0x00020000);
    const bool odd = grp & 1;
    // (the stores as non-temporal or sc1 instead of the default policy, so that the table block
    // being written would not evict the stripe the gather reads from the Infinity Cache: config-4
    // job 0.5968 / 0.5967 / 0.5966 s, base / nt / sc1 means of three interleaved runs, profiles/r5/nt)
    // Float tables: even lanes e, odd lanes e*s. Split16: even lanes the hi word (one v_perm_b32)
    // and e into the ex pair, odd lanes e*s into the pair's second word.
    const uint32_t eb = __float_as_uint(e), sb = __float_as_uint(e * sv);
    const int off2 = tab.ex ? (off < 0 ? off : 2 * off + (odd ? 4 : 0)) : (odd ? off : (int)0x80000000);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(sb, eb, tab.sel_e), re, odd ? (int)0x80000000 : off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(odd ? sb : eb, rs, off2, 0, 0);
  };

  // One unit per step, in block-major order: block m (16 hidden units) takes its KS groups of 12
  // MFMAs (KS = D / 32) into acc[m & 1], and the epilogue of the block before it (w2 . ReLU, 8
  // values per lane) runs one group later, between block m's MFMAs -- so only two blocks'
  // accumulators are live (16 VGPRs instead of a whole second unit's). Block 0's epilogue slot
  // finishes the previous unit (its last block, then its tail); the unit's own blocks 0 .. MB - 2
  // accumulate into apc. The hidden slices of cur / prev / the unit built (bu) are compile-time
  // (X6Slices): the slice's W1 registers, b1 / w2 offsets and the item's tail are fixed per call
  // site -- no selects, no branches. A fragments are read one group ahead.
  static_assert(MB % 2 == 0, "x6n: block parity is compile-time");
  floatx4 acc[2][2];
  float apc0 = 0.f, apc1 = 0.f;
  // one hidden slice (NHU == 1, no distance columns, D <= 64): this lane's S*b1 / w2/S rows of
  // every block in VGPRs, loaded once per chunk, instead of an LDS read -- and its lgkmcnt(0) wait,
  // which also drained the next group's A reads -- at every block's start and epilogue: D = H = 64
  // 197 -> 233 VGPRs, table block 1.982 -> 1.905 ms, config-4 job 0.603 -> 0.597 s interleaved
  // (profiles/r5/er). (D = 128 would spill; the distance variants sit at 245 VGPRs already.) The
  // tail's s / history-id reads and the build's history-row reads a group ahead as well: neutral
  // (block 1.863 vs 1.855 / 1.858 ms without either, job 0.5964 / 0.5958 / 0.5961 s, profiles/r5/tp).
  constexpr bool ER = X6N_EPI_REGS && NHU == 1 && !DIST && D <= 64;
  float4 breg[ER ? MB : 1], wreg[ER ? MB : 1];
  auto wld = [&](const float* ewb, int m) __attribute__((always_inline)) {
    if constexpr (ER) return wreg[m];
    else return *reinterpret_cast<const float4*>(ewb + 4 * grp);
  };
  auto epi = [&](const float4 w4, const floatx4 (&a)[2], float& t0, float& t1) __attribute__((always_inline)) {
    t0 = __builtin_fmaf(w4.x, relu_bits(a[0][0]), t0);
    t0 = __builtin_fmaf(w4.y, relu_bits(a[0][1]), t0);
    t0 = __builtin_fmaf(w4.z, relu_bits(a[0][2]), t0);
    t0 = __builtin_fmaf(w4.w, relu_bits(a[0][3]), t0);
    t1 = __builtin_fmaf(w4.x, relu_bits(a[1][0]), t1);
    t1 = __builtin_fmaf(w4.y, relu_bits(a[1][1]), t1);
    t1 = __builtin_fmaf(w4.z, relu_bits(a[1][2]), t1);
    t1 = __builtin_fmaf(w4.w, relu_bits(a[1][3]), t1);
  };
  auto step = [&](auto do_mma, auto sl, const uint4* src, int cur, int prev, bool live, int bu, int bgrp,
                  int bit) __attribute__((always_inline)) {
    constexpr bool MMA = decltype(do_mma)::value;
    constexpr int HC = decltype(sl)::cur, HPV = decltype(sl)::prev, HB = decltype(sl)::built;
    constexpr int NG = KS * MB;                 // (m, s) groups of 12 MFMAs
    constexpr int EG = KS > 1 ? 1 : 0;          // a block's epilogue slot: its successor's group EG
    const float* ebc = eb + HPU * HC;
    const float* ewc = ew + HPU * HC;
    const float* ewp = ew + HPU * HPV + 16 * (MB - 1);
    (void)cur;
    auto aload = [&](int g, half8 (&a)[3]) __attribute__((always_inline)) {
      const int m = g / KS, s = g % KS;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const uint4 u4 = src[q * NE + (m * KS + s) * 64 + lane];
        a[q] = *reinterpret_cast<const half8*>(&u4);
      }
    };
    // EP: the LDS reads of S*b1 / w2/S issued one group ahead of their use, before that group's A
    // reads, so the wait for them is a counted one that leaves the A reads in flight (where ER does
    // not apply; lgkmcnt(0) waits per hot block 22 -> 13 at D = H = 128: block 7.478 -> 7.404 ms,
    // region_distance 2.200 -> 2.180 ms, its config-4 job 0.620 -> 0.617 s, profiles/r5/ep)
    constexpr bool EP = !ER && X6N_EPI_PREFETCH;
    float4 bnx = {0.f, 0.f, 0.f, 0.f}, wnx = {0.f, 0.f, 0.f, 0.f};
    auto eload = [&](int g) __attribute__((always_inline)) {   // what group g's consumers need
      const int m = g / KS, s = g % KS;
      if (s == 0) bnx = *reinterpret_cast<const float4*>(ebc + 16 * m + 4 * grp);
      if (s == EG) wnx = *reinterpret_cast<const float4*>((m == 0 ? ewp : ewc + 16 * (m - 1)) + 4 * grp);
    };
    if constexpr (EP) {
      if (MMA) eload(0);
      else wnx = *reinterpret_cast<const float4*>(ewp + 4 * grp);   // the drain step: its epilogue only
    }
    half8 a_nx[3];
    if (MMA) aload(0, a_nx);
    if constexpr (DIST && MMA && HC == 0) {   // the item's features (formed one item ahead)
      fB0 = fN0;
      fB1 = fN1;
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int m = g / KS, s = g % KS;
      const float4 wcur = wnx;   // EP: this group's epilogue row (if it has one), read a group ago
      if (MMA) {
        if (s == 0) {   // the block's accumulators start at S*b1 (the MFMA's C operand)
          float4 b4;
          if constexpr (ER) b4 = breg[m];
          else if constexpr (EP) b4 = bnx;
          else b4 = *reinterpret_cast<const float4*>(ebc + 16 * m + 4 * grp);
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) {
            acc[m & 1][nb][0] = b4.x; acc[m & 1][nb][1] = b4.y;
            acc[m & 1][nb][2] = b4.z; acc[m & 1][nb][3] = b4.w;
          }
        }
        half8 a_[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) a_[q] = a_nx[q];
        if constexpr (EP) {
          if (g + 1 < NG) eload(g + 1);
        }
        if (g + 1 < NG) aload(g + 1, a_nx);
        acc[m & 1][0] = mfma16n_pieces(a_, tb[0][s], acc[m & 1][0]);
        acc[m & 1][1] = mfma16n_pieces(a_, tb[1][s], acc[m & 1][1]);
        if constexpr (DIST) {   // the two distance columns: one exact fp32 K-step per feature
          if ((m & 1) && s == 0) {   // blocks (m - 1, m): block m - 1's MFMAs are done, m's started
            // lane group g supplies block g = (block m - 1 + (g >> 1), candidate block g & 1)
            const float2 ad = *reinterpret_cast<const float2*>(Adn + (HPU * HC + 16 * (m - 1 + (grp >> 1)) + l16) * 4);
            floatx16 c4 = __builtin_shufflevector(
                __builtin_shufflevector(acc[0][0], acc[0][1], 0, 1, 2, 3, 4, 5, 6, 7),
                __builtin_shufflevector(acc[1][0], acc[1][1], 0, 1, 2, 3, 4, 5, 6, 7),
                0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
            c4 = mfma4b(ad.x, fB0, c4);
            c4 = mfma4b(ad.y, fB1, c4);
            acc[0][0] = __builtin_shufflevector(c4, c4, 0, 1, 2, 3);
            acc[0][1] = __builtin_shufflevector(c4, c4, 4, 5, 6, 7);
            acc[1][0] = __builtin_shufflevector(c4, c4, 8, 9, 10, 11);
            acc[1][1] = __builtin_shufflevector(c4, c4, 12, 13, 14, 15);
          }
        }
        // a unit of the next group, at the step's middle group (D = H = 128 block 7.60 -> 7.45 ms
        // against the last group; D = 64 unchanged -- profiles/r4/ab6). (Round 5 timed the kernel
        // without this build, wrong results: 1.822 of 2.050 ms per D = 64 table block, MFMA busy
        // 0.64 instead of 0.56, profiles/r5/pmc_probe; the probe switch is gone since round 6.)
        if (g == NG / 2) build(bu, std::integral_constant<int, HB>{}, bgrp, bit);
        // the next item's distance features, in the item's last unit (compile-time)
        if constexpr (DIST && HC == NHU - 1)
          if (g == std::min(X6N_FEATS_AT >= 0 ? X6N_FEATS_AT : (D <= 64 ? 3 : 1), NG - 1))
            feats(NHU == 1 ? cur + 1 : cur / NHU + 1);
      }
      if constexpr (D == 128) {
        // issue order of the group: the next group's A reads, then MFMAs with VALU between
        // (D = H = 128 block 7.60 -> 7.46 ms; at D = 64 it costs 5 %, profiles/r4/ab6; counting
        // EP's extra read into the first set where a group has one: 7.171 -> 7.275 ms, profiles/r5/sep)
        if (MMA) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          if (!MMA) break;
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
      }
      if (s != EG) continue;
      if (m == 0) {   // the previous unit's last block, then that unit is complete
        float ap0 = apc0, ap1 = apc1;
        epi(EP ? wcur : wld(ewp, MB - 1), acc[(MB - 1) & 1], ap0, ap1);
        apc0 = 0.f;
        apc1 = 0.f;
        if constexpr (NHU == 1) {
          tail(prev >= 0 ? prev : 0, ap0, ap1, live);
        } else {                 // an item's units add their partials; its last one, the tail
          pa0 = HPV == 0 ? ap0 : pa0 + ap0;
          pa1 = HPV == 0 ? ap1 : pa1 + ap1;
          if constexpr (HPV == NHU - 1) tail(prev < 0 ? 0 : prev / NHU, pa0, pa1, live);
        }
      } else if (MMA) {
        epi(EP ? wcur : wld(ewc + 16 * (m - 1), m - 1), acc[(m - 1) & 1], apc0, apc1);
      }
    }
  };

  for (j0 = 0; j0 < hlen; j0 += JCB) {
    const int jn = (int)std::min<int64_t>(JCB, hlen - j0);
    __syncthreads();   // the previous chunk's ring, hrows and hid readers are done
    float hmax = 0.f;
    for (int f = tid; f < jn * (D / 4); f += THREADS) {
      const int jj = f / (D / 4), q4 = f % (D / 4);
      const int64_t item = indices[hbeg + j0 + jj];
      float4 v;
      if (!REGION || q4 < DH / 4)
        v = reinterpret_cast<const float4*>(p.eh + item * p.item_dim)[q4];
      else
        v = reinterpret_cast<const float4*>(p.er + region_of[item] * p.region_dim)[q4 - DH / 4];
      reinterpret_cast<float4*>(hrows)[f] = v;
      hmax = fmaxf(hmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (int jj = tid; jj < jn; jj += THREADS) {
      const int64_t item = indices[hbeg + j0 + jj];
      hid[jj] = (int32_t)item;
      if (DIST && coords) {
        hco[2 * jj] = coords[2 * item];
        hco[2 * jj + 1] = coords[2 * item + 1];
      }
    }
    jn_cur = jn;
    const float Hm = block_max_n<NW>(hmax, red);   // barrier: chunk published
    const float SA = pow2_scale(Wmax * Hm);
    const float rs = SA / SAcur;                   // exact power-of-two ratio
    if constexpr (!W1G) {
#pragma unroll
      for (int h = 0; h < NHU; ++h)
#pragma unroll
        for (int q = 0; q < EPT; ++q)
#pragma unroll
          for (int x = 0; x < 8; ++x) wv[h][q][x] *= rs;
    }
    SAcur = SA;
    const float Sacc = SA * St, invS = 1.f / Sacc;
    Sd = Sacc;
    if constexpr (DIST) feats(0);   // the chunk's first item (hco / hid published above)
    for (int f = lane; f < EPI; f += 64) Escl[wave * EPI + f] = Eimg[f] * (f < HP ? Sacc : invS);
    {   // s tile of the chunk: items (pieces of h * S_h, M) x this wave's candidates (N), kept as
        // s = value / (S_h S_t) in the wave's own LDS slot, [candidate][item]
      const float Sh = pow2_scale(Hm);
      const float invShSt = 1.f / (Sh * St);
      constexpr int MI = JCB / 16;   // 16-item tiles of the chunk
      floatx4 sacc[MI][2];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) sacc[mi][nb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int it = 16 * mi + l16;
        const bool ok = it < jn;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const float* hp = hrows + it * D + 32 * s + 8 * grp;
          const float4 h0 = *reinterpret_cast<const float4*>(hp);
          const float4 h1 = *reinterpret_cast<const float4*>(hp + 4);
          float x[8];
          x[0] = ok ? h0.x * Sh : 0.f; x[1] = ok ? h0.y * Sh : 0.f;
          x[2] = ok ? h0.z * Sh : 0.f; x[3] = ok ? h0.w * Sh : 0.f;
          x[4] = ok ? h1.x * Sh : 0.f; x[5] = ok ? h1.y * Sh : 0.f;
          x[6] = ok ? h1.z * Sh : 0.f; x[7] = ok ? h1.w * Sh : 0.f;
          half8 hpc[3];
          split_pieces<3>(x, hpc);
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) sacc[mi][nb] = mfma16n_pieces(hpc, tb[nb][s], sacc[mi][nb]);
        }
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sv_mine[(16 * nb + l16) * SVP + 16 * mi + 4 * grp + r] = sacc[mi][nb][r] * invShSt;
    }
    const int nunits = jn * NHU;
    const int ngroups = (nunits + GU - 1) / GU;
    build(0, std::integral_constant<int, 0>{}, 0, 0);
    if (GU == 2 && nunits > 1) build(1, std::integral_constant<int, 1 % NHU>{}, 0, 1);
    __syncthreads();   // group 0's fragments, this wave's S*b1 / w2/S and s tile published
    if constexpr (ER) {
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        breg[m] = *reinterpret_cast<const float4*>(eb + 16 * m + 4 * grp);
        wreg[m] = *reinterpret_cast<const float4*>(ew + 16 * m + 4 * grp);
      }
    }
    // one group: its units' steps, each building a unit of the next group (past the chunk's end a
    // clamped copy nobody reads) and finishing the previous unit; groups go in rounds of GQ (ring
    // slot GP & 1), so every step's hidden slices are compile-time. With GU = 2 and an odd unit
    // count the last step runs on a stale slot: only its finish of the unit before it is used.
    auto group = [&](int g, auto gpar) __attribute__((always_inline)) {
      constexpr int GP = decltype(gpar)::value;
      constexpr int SLOT = GP & 1;
      auto one = [&](auto itc) __attribute__((always_inline)) {
        constexpr int it = decltype(itc)::value;
        constexpr int HC = (GP * GU + it) % NHU;   // u % NHU: a round spans GQ * GU units, a
                                                   // multiple of NHU (static_assert in CfgN)
        using SL = X6Slices<HC, (HC + NHU - 1) % NHU, (HC + GU) % NHU>;
        const int u = g * GU + it;
        const int bu = std::min(u + GU, nunits - 1);
        step(std::true_type{}, SL{}, ring + ((SLOT * GU + it) * 3) * NE, u, u - 1, u > 0, bu, SLOT ^ 1, it);
      };
      one(std::integral_constant<int, 0>{});
      if constexpr (GU == 2) one(std::integral_constant<int, 1>{});
      // (without this barrier, a round-5 timing probe with racing ring slots: 1.998 vs 2.050 ms
      // per D = 64 table block, profiles/r5/pmc_probe)
      __syncthreads();
    };
    for (int g = 0; g < ngroups; g += C::GQ) {
      group(g, std::integral_constant<int, 0>{});
      if (g + 1 < ngroups) group(g + 1, std::integral_constant<int, 1>{});
      if constexpr (C::GQ > 2) {
        if (g + 2 < ngroups) group(g + 2, std::integral_constant<int, 2>{});
        if (g + 3 < ngroups) group(g + 3, std::integral_constant<int, 3>{});
      }
    }
    const int last = ngroups * GU - 1;   // the last step's unit
    if (last == nunits - 1) {            // drain: the epilogue of the chunk's last unit, no MFMAs
      step(std::false_type{}, X6Slices<0, NHU - 1, 0>{}, ring, last, last, true, 0, 0, 0);
    }
  }
  if (!tab.e) {
    const float logit = finish_logit(S, N, p.beta, hlen == 0);
    const bool isnan_ = logit != logit;
    float sc = sigmoidf_ref(logit);
    if (isnan_) sc = __builtin_nanf("");
    if (in_hist) sc = -1.f;
    const bool writer = vout && !(grp & 1);
    if (writer) scores[wslot * score_ld + cout] = sc;
    if (nan_count) {
      const unsigned long long m = __ballot(writer && !in_hist && isnan_);
      if (lane == 0 && m) atomicAdd(nan_count, (int32_t)__popcll(m));
    }
  }
  }
}

// ---------------------------------------------------------------------------------------------
// Top-k per user (validation.py:26-27): exact radix select on 64-bit keys
//   key = ordered(score) << 32 | (0xFFFFFFFF - poi)   -> unique; larger key = (higher score, lower id)
// MSB-first 8-bit passes over the user's score row until the keys at or above the selected prefix
// fit a 4096-key LDS buffer (typically 2 passes), then those keys are collected and bitonic-sorted
// in LDS and the first k kept. NaN (canonical, positive) orders above +inf.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ord_f32(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// Visit (c, score) for every c in [0, P): 16-byte loads when the row is 16-byte aligned.
template <class F>
__device__ __forceinline__ void topk_visit(const float* __restrict__ s, int64_t P, F&& f) {
  const int tid = threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(s) & 15) == 0) {
    const int64_t P4 = P >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(s);
#pragma unroll 2
    for (int64_t q = tid; q < P4; q += TOPK_THREADS) {
      const float4 v = s4[q];
      f(4 * q, v.x);
      f(4 * q + 1, v.y);
      f(4 * q + 2, v.z);
      f(4 * q + 3, v.w);
    }
    for (int64_t c = 4 * P4 + tid; c < P; c += TOPK_THREADS) f(c, s[c]);
  } else {
    for (int64_t c = tid; c < P; c += TOPK_THREADS) f(c, s[c]);
  }
}

// LDS histogram add with the wave's most common bin (the first active lane's) added once by one
// lane: score rows cluster in a few top digits, and same-address LDS atomics serialise.
__device__ __forceinline__ void topk_hist_add(uint32_t* hist, bool pred, uint32_t bin) {
  const unsigned long long act = __ballot(pred);
  if (!act) return;
  const int leader = __ffsll((long long)act) - 1;
  const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, leader);
  const unsigned long long same = __ballot(pred && bin == b0);
  if ((int)(threadIdx.x & 63) == leader) atomicAdd(&hist[b0], (uint32_t)__popcll(same));
  else if (pred && bin != b0) atomicAdd(&hist[bin], 1u);
}

constexpr int TOPK_CAP = 4096;   // keys collected for the final sort (32 KiB of LDS)

__global__ void __launch_bounds__(TOPK_THREADS)
topk_kernel(const float* __restrict__ scores, int64_t score_ld, int64_t P, int k,
            int32_t* __restrict__ out_ids, float* __restrict__ out_scores,
            int32_t* __restrict__ short_count) {
  __shared__ uint32_t hist[256];
  __shared__ unsigned long long buf[TOPK_CAP];
  __shared__ uint32_t sh_bin, sh_above, sh_binc, sh_total, sh_cnt;
  const float* s = scores + (int64_t)blockIdx.x * score_ld;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long prefix = 0, mask = 0;
  uint32_t rem = (uint32_t)k, above_total = 0, n_collect = 0;
  int kk = k;
  // MSB-first 8-bit digits of the 64-bit key; stop as soon as the keys at or above the selected
  // digit prefix (the k winners plus the rest of their bin) fit the collect buffer -- usually
  // after the second digit -- so a row is read 3 times instead of 9.
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    topk_visit(s, P, [&](int64_t c, float v) {
      const bool cand = !(v < 0.f);   // history POI (or padding) = -1: not a candidate
      const unsigned long long key =
          ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)c);
      topk_hist_add(hist, cand && (key & mask) == prefix, (uint32_t)(key >> shift) & 255u);
    });
    __syncthreads();
    if (wave == 0) {
      const int base = 255 - lane * 4;
      const uint32_t c0 = hist[base], c1 = hist[base - 1], c2 = hist[base - 2], c3 = hist[base - 3];
      const uint32_t local = c0 + c1 + c2 + c3;
      uint32_t incl = local;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      const uint32_t total = __shfl(incl, 63);
      if (pass == 0 && lane == 0) sh_total = total;
      uint32_t need = rem;
      if (pass == 0 && total < need) need = total;  // fewer candidates than k
      const uint32_t excl = incl - local;
      if (need > 0 && excl < need && incl >= need) {
        uint32_t cum = excl;
        int bsel;
        uint32_t bc;
        if (cum + c0 >= need) { bsel = base; bc = c0; }
        else if ((cum += c0) + c1 >= need) { bsel = base - 1; bc = c1; }
        else if ((cum += c1) + c2 >= need) { bsel = base - 2; bc = c2; }
        else { cum += c2; bsel = base - 3; bc = c3; }
        sh_bin = (uint32_t)bsel;
        sh_above = cum;
        sh_binc = bc;
      }
      if (need == 0 && lane == 0) { sh_bin = 0; sh_above = 0; sh_binc = 0; }
    }
    __syncthreads();
    if (pass == 0) {
      if (sh_total < (uint32_t)kk) kk = (int)sh_total;
      rem = (uint32_t)kk;
    }
    prefix |= (unsigned long long)sh_bin << shift;
    mask |= 255ull << shift;
    rem -= sh_above;
    above_total += sh_above;
    n_collect = above_total + sh_binc;   // keys >= prefix
    __syncthreads();
    if (kk == 0 || n_collect <= (uint32_t)TOPK_CAP) break;   // block-uniform
  }
  if (tid == 0) sh_cnt = 0;
  __syncthreads();
  if (kk > 0) {
    topk_visit(s, P, [&](int64_t c, float v) {
      if (v < 0.f) return;
      const unsigned long long key =
          ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)c);
      if (key >= prefix) {
        const uint32_t pos = atomicAdd(&sh_cnt, 1u);
        if (pos < (uint32_t)TOPK_CAP) buf[pos] = key;
      }
    });
  } else {
    n_collect = 0;
  }
  __syncthreads();
  int n2 = 1;
  while (n2 < (int)n_collect || n2 < k) n2 <<= 1;
  for (int i = (int)n_collect + tid; i < n2; i += TOPK_THREADS) buf[i] = 0ull;   // keys > 0
  __syncthreads();
  // bitonic sort, descending; keys are unique, so the order is (score desc, id asc)
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += TOPK_THREADS) {
        const int partner = i ^ stride;
        if (partner > i) {
          const bool desc = (i & size) == 0;
          const unsigned long long x = buf[i], y = buf[partner];
          if (desc ? (x < y) : (x > y)) {
            buf[i] = y;
            buf[partner] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += TOPK_THREADS) {
    int32_t id = -1;
    float sc = __builtin_nanf("");
    if (i < kk) {
      const unsigned long long key = buf[i];
      id = (int32_t)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
      sc = unord_f32((uint32_t)(key >> 32));
    }
    out_ids[(int64_t)blockIdx.x * k + i] = id;
    out_scores[(int64_t)blockIdx.x * k + i] = sc;
  }
  if (tid == 0 && kk < k && short_count) atomicAdd(short_count, 1);
}

// ---------------------------------------------------------------------------------------------
// Power-law geo prior (powerLaw.py:7-21, 86-92) and its blend (run.py:55-59, 537-539).
// float64 throughout, in the reference's operation order; every product/sum is an explicit
// round-to-nearest op (__dmul_rn / __dadd_rn / __dsub_rn) so the compiler cannot contract FMAs.
// Per POI: phi = (90 - lat) * d2r, theta = lng * d2r (d2r = math.pi / 180.0).
// ---------------------------------------------------------------------------------------------
// Geo, make_geo, ref_dist: nais_geo.h

// ref_pr_d (PowerLaw.pr_d): nais_geo.h
constexpr int PRIOR_THREADS = 256;
constexpr int PRIOR_JC = 256;

// G[slot][c] = prod_j pr_d(dist(coo_j, coo_c)) over the user's history in CSR order
// (np.prod, powerLaw.py:92); history POIs get -1. gmax[slot] = max over candidates (u64 bits).
// zero_exit (prior_zero_exit(a, b)): long histories underflow G to 0.0 after ~110 POIs at city
// distances; the remaining factors are then not evaluated (bit-identical, see the loop).
__global__ void __launch_bounds__(PRIOR_THREADS)
prior_kernel(const double* __restrict__ coords, int64_t P, const int64_t* __restrict__ indptr,
             const int64_t* __restrict__ indices, const int32_t* __restrict__ users, double pa,
             double pb, double* __restrict__ G, int64_t ld, unsigned long long* __restrict__ gmax,
             int zero_exit) {
  __shared__ Geo hg[PRIOR_JC];
  __shared__ int32_t hid[PRIOR_JC];
  __shared__ double red[PRIOR_THREADS / 64];
  const int tid = threadIdx.x;
  const int64_t u = users[blockIdx.y];
  const int64_t hbeg = indptr[u], hlen = indptr[u + 1] - hbeg;
  const int64_t c = (int64_t)blockIdx.x * PRIOR_THREADS + tid;
  const bool valid = c < P;
  const int64_t cc = valid ? c : P - 1;
  const Geo gc = make_geo(coords[2 * cc], coords[2 * cc + 1]);
  double g = 1.0;
  bool in_hist = false;
  for (int64_t j0 = 0; j0 < hlen; j0 += PRIOR_JC) {
    const int jn = (int)std::min<int64_t>(PRIOR_JC, hlen - j0);
    __syncthreads();
    for (int jj = tid; jj < jn; jj += PRIOR_THREADS) {
      const int64_t item = indices[hbeg + j0 + jj];
      hid[jj] = (int32_t)item;
      hg[jj] = make_geo(coords[2 * item], coords[2 * item + 1]);
    }
    __syncthreads();
    for (int jj = 0; jj < jn; ++jj) {
      // zero_exit: a product that reached +0.0 stays +0.0 (every factor finite and >= +0), so
      // the f64 haversine + pow is skipped -- for the whole wave once all its lanes are there
      if (!zero_exit || g != 0.0) g = __dmul_rn(g, ref_pr_d(pa, pb, ref_dist(hg[jj], gc)));
      in_hist |= hid[jj] == (int32_t)c;
    }
  }
  if (hlen == 0) g = 1.0;   // np.prod([]) == 1.0
  if (valid) G[(int64_t)blockIdx.y * ld + c] = in_hist ? -1.0 : g;
  double m = (valid && !in_hist) ? g : -1.0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    double mm = red[0];
    for (int w = 1; w < PRIOR_THREADS / 64; ++w) mm = fmax(mm, red[w]);
    if (mm >= 0.0) atomicMax(gmax + blockIdx.y, (unsigned long long)__double_as_longlong(mm));
  }
}

// blended score of candidate c (run.py:537-539 with normalize run.py:55-59):
//   (1 - alpha) * pred  in float32 (torch: f32 tensor * python scalar), then + alpha * G_norm in f64
__device__ __forceinline__ bool blended(const float* s, const double* g, double gm, float om_alpha_f,
                                        double alpha, int64_t c, double& out) {
  const float v = s[c];
  if (v < 0.f) return false;                       // history POI: not a candidate
  const double gn = (gm != 0.0) ? __ddiv_rn(g[c], gm) : g[c];
  out = __dadd_rn((double)(v * om_alpha_f), __dmul_rn(alpha, gn));
  return true;
}

__device__ __forceinline__ unsigned long long ord_f64(double d) {
  unsigned long long u = (unsigned long long)__double_as_longlong(d);
  if (d != d) u = 0x7ff8000000000000ull;           // canonical NaN ranks first (torch.topk)
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double unord_f64(unsigned long long o) {
  const unsigned long long u = (o & 0x8000000000000000ull) ? (o & 0x7fffffffffffffffull) : ~o;
  return __longlong_as_double((long long)u);
}

// top-k over the f64 blended scores: radix select on the 64-bit ordered score, MSB-first 8-bit
// digits, stopping as soon as the candidates at or above the selected prefix fit the collect
// buffer (after 2-3 digits for scores spread over (0, 1): the row -- 12 B and one f64 division per
// candidate -- is read 3-4 times instead of 13); only when more than BLEND_CAP candidates share the whole 64-bit score
// does it go on to the ~id digits among the scores equal to the threshold (4 passes). Then
// collect and bitonic-sort by (score, ~id).
constexpr int BLEND_CAP = 4096;
__global__ void __launch_bounds__(TOPK_THREADS)
topk_blend_kernel(const float* __restrict__ scores, int64_t score_ld, const double* __restrict__ G,
                  int64_t g_ld, const unsigned long long* __restrict__ gmax, int64_t P, int k,
                  float om_alpha_f, double alpha, int32_t* __restrict__ out_ids,
                  float* __restrict__ out_scores, int32_t* __restrict__ short_count,
                  double* __restrict__ out_blend) {
  __shared__ uint32_t hist[256];
  __shared__ unsigned long long bs[BLEND_CAP];
  __shared__ uint32_t bi[BLEND_CAP];
  __shared__ uint32_t sh_bin, sh_above, sh_binc, sh_total, sh_cnt;
  static_assert(BLEND_CAP >= MAX_K, "the id passes collect exactly k keys");
  const float* s = scores + (int64_t)blockIdx.x * score_ld;
  const double* g = G + (int64_t)blockIdx.x * g_ld;
  const double gm = __longlong_as_double((long long)gmax[blockIdx.x]);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long prefix = 0, mask = 0;       // over the score key
  uint32_t iprefix = 0, imask = 0;               // over ~id, among score == threshold
  uint32_t rem = (uint32_t)k, above_total = 0, n_collect = 0;
  bool early = false;                            // stopped on a score digit: collect key >= prefix
  int kk = k;
  for (int pass = 0; pass < 12; ++pass) {
    const bool idpass = pass >= 8;
    const int shift = idpass ? 24 - 8 * (pass - 8) : 56 - 8 * pass;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int64_t c0 = 0; c0 < P; c0 += TOPK_THREADS) {   // block-uniform trip count (ballots)
      const int64_t c = c0 + tid;
      double v = 0.0;
      const bool ok = c < P && blended(s, g, gm, om_alpha_f, alpha, c, v);
      const unsigned long long key = ord_f64(v);
      bool pred;
      uint32_t bin;
      if (!idpass) {
        pred = ok && (key & mask) == prefix;
        bin = (uint32_t)(key >> shift) & 255u;
      } else {
        const uint32_t ik = 0xFFFFFFFFu - (uint32_t)c;
        pred = ok && key == prefix && (ik & imask) == iprefix;
        bin = (ik >> shift) & 255u;
      }
      topk_hist_add(hist, pred, bin);
    }
    __syncthreads();
    if (wave == 0) {
      const int base = 255 - lane * 4;
      const uint32_t c0 = hist[base], c1 = hist[base - 1], c2 = hist[base - 2], c3 = hist[base - 3];
      const uint32_t local = c0 + c1 + c2 + c3;
      uint32_t incl = local;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      const uint32_t total = __shfl(incl, 63);
      if (pass == 0 && lane == 0) sh_total = total;
      uint32_t need = rem;
      if (pass == 0 && total < need) need = total;
      const uint32_t excl = incl - local;
      if (need > 0 && excl < need && incl >= need) {
        uint32_t cum = excl;
        int bsel;
        uint32_t bc;
        if (cum + c0 >= need) { bsel = base; bc = c0; }
        else if ((cum += c0) + c1 >= need) { bsel = base - 1; bc = c1; }
        else if ((cum += c1) + c2 >= need) { bsel = base - 2; bc = c2; }
        else { cum += c2; bsel = base - 3; bc = c3; }
        sh_bin = (uint32_t)bsel;
        sh_above = cum;
        sh_binc = bc;
      }
      if (need == 0 && lane == 0) { sh_bin = 0; sh_above = 0; sh_binc = 0; }
    }
    __syncthreads();
    if (pass == 0) {
      if (sh_total < (uint32_t)kk) kk = (int)sh_total;
      rem = (uint32_t)kk;
    }
    if (!idpass) {
      prefix |= (unsigned long long)sh_bin << shift;
      mask |= 255ull << shift;
      above_total += sh_above;
      n_collect = above_total + sh_binc;         // candidates with key >= prefix
    } else {
      iprefix |= sh_bin << shift;
      imask |= 255u << shift;
    }
    rem -= sh_above;
    __syncthreads();
    if (kk == 0) break;                                            // block-uniform
    if (!idpass && n_collect <= (uint32_t)BLEND_CAP) { early = true; break; }
  }
  if (tid == 0) sh_cnt = 0;
  __syncthreads();
  if (kk > 0) {
    for (int64_t c = tid; c < P; c += TOPK_THREADS) {
      double v;
      if (!blended(s, g, gm, om_alpha_f, alpha, c, v)) continue;
      const unsigned long long key = ord_f64(v);
      const uint32_t ik = 0xFFFFFFFFu - (uint32_t)c;
      if (early ? key >= prefix : (key > prefix || (key == prefix && ik >= iprefix))) {
        const uint32_t pos = atomicAdd(&sh_cnt, 1u);
        if (pos < (uint32_t)BLEND_CAP) {
          bs[pos] = key;
          bi[pos] = ik;
        }
      }
    }
  }
  __syncthreads();
  const int n = kk == 0 ? 0 : (early ? (int)n_collect : kk);
  int n2 = 1;
  while (n2 < n || n2 < k) n2 <<= 1;
  for (int i = n + tid; i < n2; i += TOPK_THREADS) {   // keys of real candidates are > 0
    bs[i] = 0ull;
    bi[i] = 0u;
  }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += TOPK_THREADS) {
        const int partner = i ^ stride;
        if (partner > i) {
          const bool desc = (i & size) == 0;
          const unsigned long long x = bs[i], y = bs[partner];
          const uint32_t xi = bi[i], yi = bi[partner];
          const bool less = (x < y) || (x == y && xi < yi);
          const bool greater = (x > y) || (x == y && xi > yi);
          if (desc ? less : greater) {
            bs[i] = y;
            bs[partner] = x;
            bi[i] = yi;
            bi[partner] = xi;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += TOPK_THREADS) {
    int32_t id = -1;
    double v = __builtin_nan("");
    if (i < kk) {
      id = (int32_t)(0xFFFFFFFFu - bi[i]);
      v = unord_f64(bs[i]);
    }
    out_ids[(int64_t)blockIdx.x * k + i] = id;
    out_scores[(int64_t)blockIdx.x * k + i] = (float)v;
    if (out_blend) out_blend[(int64_t)blockIdx.x * k + i] = v;   // the f64 ranking key itself
  }
  if (tid == 0 && kk < k && short_count) atomicAdd(short_count, 1);
}

// Merge of per-column-block top-k lists ranked on f64 blended scores (the column-sharded prior
// route, sharding.distributed_topk_pairs): row r holds m candidates (keys[r*m + i] f64, ids[r*m + i]
// global POI ids, id < 0 = padding); out = the k best by (key desc, id asc), NaN first -- the
// order topk_blend_kernel gives one whole row. One workgroup per row, bitonic sort in LDS.
constexpr int MERGE_THREADS = 256, MERGE_CAP = 2048;
__global__ void __launch_bounds__(MERGE_THREADS)
topk_merge_f64_kernel(const double* __restrict__ keys, const int64_t* __restrict__ ids, int m, int k,
                      int64_t* __restrict__ out_ids, float* __restrict__ out_scores,
                      double* __restrict__ out_keys) {
  __shared__ unsigned long long sk[MERGE_CAP];
  __shared__ long long si[MERGE_CAP];
  const int tid = threadIdx.x;
  const int64_t r = blockIdx.x;
  int n2 = 1;
  while (n2 < m) n2 <<= 1;
  for (int i = tid; i < n2; i += MERGE_THREADS) {
    unsigned long long key = 0ull;                 // padding: below every real key (> 0)
    long long id = 0x7fffffffffffffffll;
    if (i < m) {
      const long long x = ids[r * m + i];
      if (x >= 0) {
        key = ord_f64(keys[r * m + i]);
        id = x;
      }
    }
    sk[i] = key;
    si[i] = id;
  }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += MERGE_THREADS) {
        const int partner = i ^ stride;
        if (partner > i) {
          const bool desc = (i & size) == 0;
          const unsigned long long x = sk[i], y = sk[partner];
          const long long xi = si[i], yi = si[partner];
          // "better" = larger key, then smaller id
          const bool x_worse = (x < y) || (x == y && xi > yi);
          const bool x_better = (x > y) || (x == y && xi < yi);
          if (desc ? x_worse : x_better) {
            sk[i] = y;
            sk[partner] = x;
            si[i] = yi;
            si[partner] = xi;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += MERGE_THREADS) {
    const bool ok = i < n2 && sk[i] != 0ull;
    const double v = ok ? unord_f64(sk[i]) : __builtin_nan("");
    out_ids[r * k + i] = ok ? (int64_t)si[i] : -1;
    out_scores[r * k + i] = (float)v;
    if (out_keys) out_keys[r * k + i] = v;
  }
}

// Distance histogram for PowerLaw.fit_distance_distribution (powerLaw.py:41-55): every pair
// i < j of every user's history (CSR order), bin = int(dist(coo_i, coo_j)) (truncation, km).
constexpr int HIST_LDS_BINS = 4096;
__global__ void __launch_bounds__(256)
distance_histogram_kernel(const double* __restrict__ coords, const int64_t* __restrict__ indptr,
                          const int64_t* __restrict__ indices, int64_t num_users,
                          unsigned long long* __restrict__ hist, int64_t nbins,
                          unsigned long long* __restrict__ overflow) {
  __shared__ uint32_t lh[HIST_LDS_BINS];
  const int tid = threadIdx.x;
  const int lb = (int)std::min<int64_t>(nbins, HIST_LDS_BINS);
  for (int i = tid; i < lb; i += 256) lh[i] = 0;
  __syncthreads();
  for (int64_t u = blockIdx.x; u < num_users; u += gridDim.x) {
    const int64_t b = indptr[u], n = indptr[u + 1] - b;
    const int64_t npairs = n * (n - 1) / 2;
    for (int64_t pidx = tid; pidx < npairs; pidx += 256) {
      // pair index -> (i, j), i < j, row-major over the strict upper triangle
      int64_t i = (int64_t)((2.0 * n - 1.0 - sqrt((2.0 * n - 1.0) * (2.0 * n - 1.0) - 8.0 * (double)pidx)) / 2.0);
      if (i < 0) i = 0;
      while (i > 0 && i * (2 * n - i - 1) / 2 > pidx) --i;
      while ((i + 1) * (2 * n - i - 2) / 2 <= pidx) ++i;
      const int64_t j = pidx - i * (2 * n - i - 1) / 2 + i + 1;
      const int64_t li = indices[b + i], lj = indices[b + j];
      const Geo gi = make_geo(coords[2 * li], coords[2 * li + 1]);
      const Geo gj = make_geo(coords[2 * lj], coords[2 * lj + 1]);
      const double d = ref_dist(gi, gj);
      if (!(d >= 0.0) || d >= (double)nbins) {   // NaN or beyond the table
        atomicAdd(overflow, 1ull);
        continue;
      }
      const int64_t bin = (int64_t)d;
      if (bin < lb) atomicAdd(&lh[bin], 1u);
      else atomicAdd(hist + bin, 1ull);
    }
  }
  __syncthreads();
  for (int i = tid; i < lb; i += 256)
    if (lh[i]) atomicAdd(hist + i, (unsigned long long)lh[i]);
}

// ---------------------------------------------------------------------------------------------
// Standalone row gather (HBM roofline kernel): 16 B per lane, one row per dim/4 lanes.
// ---------------------------------------------------------------------------------------------
// Each thread moves one float4 piece per iteration; rows are read once and written once, so both
// sides use non-temporal (streaming) accesses.
typedef float nf4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256)
gather_rows_kernel(const nf4* __restrict__ table, int q4, const int64_t* __restrict__ idx,
                   int64_t m, nf4* __restrict__ out) {
  constexpr int U = 1;
  const int64_t total = m * q4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < total; i += U * stride) {
    nf4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = i + u * stride;
      const int64_t row = e / q4;
      v[u] = __builtin_nontemporal_load(table + idx[row] * q4 + (e - row * q4));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], out + i + u * stride);
  }
  for (; i < total; i += stride) {
    const int64_t row = i / q4;
    out[i] = table[idx[row] * q4 + (i - row * q4)];
  }
}

__global__ void __launch_bounds__(256)
gather_rows_scalar_kernel(const float* __restrict__ table, int dim, const int64_t* __restrict__ idx,
                          int64_t m, float* __restrict__ out) {
  const int64_t total = m * dim;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / dim;
    out[i] = table[idx[row] * dim + (i - row * dim)];
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(NAIS_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return NAIS_OK;
}

struct Shape {
  int DH, HB;
  // the generic-shape kernels (nais_generic.hip) instead of the tuned ones: nais_forward (fwd),
  // nais_score_catalog / nais_score_topk (cat), nais_pair_table (tab)
  bool gen_fwd, gen_cat, gen_tab;
};

int validate(const nais_params_t* p, Shape* sh) {
  if (!p) return fail(NAIS_E_INVALID, "params is NULL");
  if (p->variant < 0 || p->variant > 3) return fail(NAIS_E_INVALID, "unknown variant");
  if (p->precision < NAIS_PRECISION_FP32 || p->precision > NAIS_PRECISION_FP16X6_PAIRSPLIT)
    return fail(NAIS_E_INVALID, "unknown precision");
  if (!p->embed_history || !p->embed_target || !p->w1 || !p->b1 || !p->w2)
    return fail(NAIS_E_INVALID, "missing parameter pointer");
  if (p->num_pois <= 0) return fail(NAIS_E_INVALID, "num_pois must be > 0");
  if (p->num_pois > 65535ll * 256) return fail(NAIS_E_UNSUPPORTED, "num_pois > 16.7M (grid.y limit)");
  const int D = p->embed_dim;
  if (D <= 0 || D > 256)
    return fail(NAIS_E_UNSUPPORTED, "embed_dim must be in [1, 256] (the generic kernels' LDS budget)");
  if (p->hidden <= 0) return fail(NAIS_E_UNSUPPORTED, "hidden must be >= 1");
  if (p->variant == NAIS_VARIANT_BASIC) {
    if (p->item_dim != D || p->din != D) return fail(NAIS_E_INVALID, "basic: item_dim == din == embed_dim");
  } else if (p->variant == NAIS_VARIANT_DISTANCE) {
    if (p->item_dim != D || p->din != D + 2)
      return fail(NAIS_E_INVALID, "distance: item_dim == embed_dim, din == embed_dim + 2");
    if (!p->dist_w || !p->dist_b) return fail(NAIS_E_INVALID, "distance needs dist_layer weight and bias");
  } else {
    if (D % 2 != 0 || p->item_dim != D / 2 || p->region_dim != D / 2)
      return fail(NAIS_E_INVALID, "region variants: item_dim == region_dim == embed_dim/2");
    if (!p->embed_region || p->num_regions <= 0) return fail(NAIS_E_INVALID, "missing embed_region");
    const int want = D + (p->variant == NAIS_VARIANT_REGION_DISTANCE ? 2 : 0);
    if (p->din != want) return fail(NAIS_E_INVALID, "din mismatch for variant");
    if (p->variant == NAIS_VARIANT_REGION_DISTANCE && (!p->dist_w || !p->dist_b))
      return fail(NAIS_E_INVALID, "region_distance needs dist_layer weight and bias");
  }
  // the tuned kernels: embed widths 8 / 16 / 32 / 64 / 128 (the MFMA K tiles), hidden <= 256 in
  // the forward and the fp16x6 item-side kernel (D 32 / 64 / 128), <= 128 in the other catalog
  // kernels; every other shape takes the generic kernels (exact fp32)
  const bool native = D == 8 || D == 16 || D == 32 || D == 64 || D == 128;
  const bool x6n = D == 32 || D == 64 || D == 128;
  sh->gen_fwd = !native || p->hidden > 256;
  sh->gen_cat = sh->gen_fwd || (p->hidden > 128 && !(x6n && p->precision == NAIS_PRECISION_FP16X6));
  sh->gen_tab = sh->gen_fwd || (p->hidden > 128 && !(x6n && (p->precision == NAIS_PRECISION_FP16X6 ||
                                                            p->precision == NAIS_PRECISION_FP16X6_PAIRSPLIT)));
  sh->DH = native ? D / 2 : 4;
  int hb = (p->hidden + 31) / 32;   // 32-hidden blocks: 1, 2, 4 or 8 (hidden > 128)
  if (hb == 3) hb = 4;
  if (hb > 4) hb = 8;
  sh->HB = hb;
  return NAIS_OK;
}

int to_dev(const nais_params_t* p, DevParams* d) {
  d->eh = p->embed_history;
  d->et = p->embed_target;
  d->er = p->embed_region;
  d->w1 = p->w1;
  d->b1 = p->b1;
  d->w2 = p->w2;
  d->P = p->num_pois;
  d->item_dim = p->item_dim;
  d->region_dim = p->region_dim;
  d->H = p->hidden;
  d->din = p->din;
  d->beta = p->beta;
  d->wd = p->dist_w;
  d->bd = p->dist_b;
  return NAIS_OK;
}

template <int DH, int HB, int VAR>
size_t catalog_lds() {
  constexpr bool DIST = VarT<VAR>::DIST;
  return Consts<DH, HB, DIST>::BYTES + size_t(JC) * 2 * DH * 4 + size_t(JC) * 4 +
         (DIST ? size_t(JC) * 16 : 0);
}

template <int DH, int HB, int VAR>
int launch_catalog(const DevParams& d, const int64_t* indptr, const int64_t* indices,
                   const int32_t* users, int nb, const int64_t* region_of, const double* coords,
                   const double* latlon_mat, float* scores, int64_t ld, int32_t* nan_count,
                   hipStream_t stream, const TableOut& tab = TableOut{}) {
  if constexpr (HB > 4) {
    return fail(NAIS_E_UNSUPPORTED, "hidden > 128: the catalog kernels take it at precision fp16x6 "
                                    "with embed_dim 32, 64 or 128");
  } else {
  const size_t lds = catalog_lds<DH, HB, VAR>();
  auto kern = catalog_score_kernel<DH, HB, VAR>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  dim3 grid = tab.e ? table_grid(tab, nb) : cat_grid(d.P, nb, CAND_PER_BLOCK);
  hipLaunchKernelGGL(kern, grid, dim3(THREADS), lds, stream, d, indptr, indices, users, region_of,
                     coords, latlon_mat, scores, ld, nan_count, tab);
  return check_launch("catalog_score_kernel");
  }
}

constexpr size_t kLdsBytes = 160 * 1024;   // LDS per workgroup on gfx950 (MI355X_MICROARCH.md)

template <int DH, int HB, int VAR, int NPC>
size_t catalog_x3_lds() {
  constexpr bool DIST = VarT<VAR>::DIST;
  return Consts16<DH, HB, DIST, NPC>::BYTES + size_t(JC) * 2 * DH * 4 + size_t(JC) * 4 +
         (DIST ? size_t(JC) * 16 : 0);
}

template <int DH, int HB, int VAR, int NPC = 2>
int launch_catalog_x3(const DevParams& d, const int64_t* indptr, const int64_t* indices,
                      const int32_t* users, int nb, const int64_t* region_of, const double* coords,
                      const double* latlon_mat, float* scores, int64_t ld, int32_t* nan_count,
                      hipStream_t stream, const TableOut& tab = TableOut{}) {
  if constexpr (DH % 8 != 0 || HB > 4) {  // D = 8: one K=16 f16 step would be half padding; use fp32
    return launch_catalog<DH, HB, VAR>(d, indptr, indices, users, nb, region_of, coords, latlon_mat,
                                       scores, ld, nan_count, stream, tab);
  } else {
    const size_t lds = catalog_x3_lds<DH, HB, VAR, NPC>();
    if (lds > kLdsBytes) return fail(NAIS_E_INVALID, "catalog_score_x3_kernel: shape exceeds LDS");
    auto kern = catalog_score_x3_kernel<DH, HB, VAR, NPC>;
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
    dim3 grid = tab.e ? table_grid(tab, nb) : cat_grid(d.P, nb, CAND_PER_BLOCK);
    hipLaunchKernelGGL(kern, grid, dim3(THREADS), lds, stream, d, indptr, indices, users, region_of,
                       coords, latlon_mat, scores, ld, nan_count, tab);
    return check_launch("catalog_score_x3_kernel");
  }
}

// the 16x16x32 item-side kernel (x6n) instead of x3b / the per-pair split kernel for every fp16x6
// shape it covers: D in {32, 64, 128}, H <= 256, every variant (the distance variants since round 5).
// Round-4 A/B against x3b at config 4: standalone 512-column table block 2.179 -> 1.990 ms, the job
// 623 -> 601 ms (profiles/r4/x6n); at D = H = 128 against the per-pair split kernel: config-5 direct
// 6.35e7 -> 7.32e7 pairs/s (profiles/r4/d128). The A/B switch is gone; x3b keeps fp16x3.
template <int DH, int HB, int VAR, int NPC = 2>
int launch_catalog_x3b(const DevParams& d, const int64_t* indptr, const int64_t* indices,
                       const int32_t* users, int nb, const int64_t* region_of, const double* coords,
                       const double* latlon_mat, float* scores, int64_t ld, int32_t* nan_count,
                       hipStream_t stream, const TableOut& tab = TableOut{}) {
  if constexpr (NPC == 3 && (DH == 16 || DH == 32 || DH == 64)) {
    // one unit up to 64 hidden units, two at H = 128 (D = 128 with 32-hidden units, MB = 2:
    // 1 % slower in the same process, profiles/r4/ab8)
    constexpr int D = 2 * DH;
    constexpr int MB = HB <= 2 ? 2 * HB : 4;
    constexpr int NHU = HB <= 2 ? 1 : HB / 2;   // 64-hidden units: 2 at H <= 128, 4 at H <= 256
    using CN = CfgN<D, MB, NHU, VarT<VAR>::DIST>;
    const size_t lds = CN::BYTES;
    auto kern = catalog_score_x6n_kernel<D, MB, NHU, VAR>;
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
    dim3 grid = tab.e ? table_grid(tab, nb, CN::CPB) : cat_grid(d.P, nb, CN::CPB);
    TableOut t = tab;
    if (t.e && t.work) {   // work queue: one workgroup per CU of the stream's mask (the LDS
      t.ngroups = (int32_t)grid.y;   // holds one), items tile-major
      t.ntiles = (int32_t)grid.x;
      const int ncu = nais_internal_stream_cus(stream);
      if (ncu <= 0) return fail(NAIS_E_HIP, "device attributes");
      grid = dim3((unsigned)std::min<int64_t>((int64_t)grid.x * grid.y, ncu), 1, 1);
      if (hipMemsetAsync(t.work, 0, sizeof(int32_t), stream) != hipSuccess)
        return fail(NAIS_E_HIP, "hipMemsetAsync(work)");
    } else {
      t.work = nullptr;
    }
    hipLaunchKernelGGL(kern, grid, dim3(CN::THREADS), lds, stream, d, indptr, indices, users,
                       region_of, coords, latlon_mat, scores, ld, nan_count, t);
    return check_launch("catalog_score_x6n_kernel");
  } else if constexpr (HB > 4) {
    return fail(NAIS_E_UNSUPPORTED, "hidden > 128: the catalog kernels take it at precision fp16x6 "
                                    "with embed_dim 32, 64 or 128");
  } else if constexpr (DH % 8 != 0) {
    return launch_catalog<DH, HB, VAR>(d, indptr, indices, users, nb, region_of, coords, latlon_mat,
                                       scores, ld, nan_count, stream, tab);
  } else if constexpr ((VarT<VAR>::DIST && !CfgB<DH, HB, true, WAVES, NPC>::PIPE) ||
                       CfgB<DH, HB, false, WAVES, NPC>::BYTES > kLdsBytes) {
    // the distance features ride on the per-pair split kernel (also in pair-table mode) except on
    // the pipelined item-side shapes (D, H <= 64), whose step adds them as one exact fp32 MFMA
    // K-step; so do shapes whose item ring does not fit the LDS (fp16x6 at D = H = 128)
    return launch_catalog_x3<DH, HB, VAR, NPC>(d, indptr, indices, users, nb, region_of, coords,
                                               latlon_mat, scores, ld, nan_count, stream, tab);
  } else {
    constexpr int NW = WAVES;
    const size_t lds = CfgB<DH, HB, VarT<VAR>::DIST, NW, NPC>::BYTES;
    auto kern = catalog_score_x3b_kernel<DH, HB, VAR, NW, NPC>;
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
    dim3 grid = tab.e ? table_grid(tab, nb, NW * 32) : cat_grid(d.P, nb, NW * 32);
    hipLaunchKernelGGL(kern, grid, dim3(NW * 64), lds, stream, d, indptr, indices, users, region_of,
                       coords, latlon_mat, scores, ld, nan_count, tab);
    return check_launch("catalog_score_x3b_kernel");
  }
}

template <int DH, int HB, int VAR>
int launch_catalog_x6b(const DevParams& d, const int64_t* indptr, const int64_t* indices,
                       const int32_t* users, int nb, const int64_t* region_of, const double* coords,
                       const double* latlon_mat, float* scores, int64_t ld, int32_t* nan_count,
                       hipStream_t stream, const TableOut& tab = TableOut{}) {
  return launch_catalog_x3b<DH, HB, VAR, 3>(d, indptr, indices, users, nb, region_of, coords,
                                            latlon_mat, scores, ld, nan_count, stream, tab);
}
template <int DH, int HB, int VAR>
int launch_catalog_x6(const DevParams& d, const int64_t* indptr, const int64_t* indices,
                      const int32_t* users, int nb, const int64_t* region_of, const double* coords,
                      const double* latlon_mat, float* scores, int64_t ld, int32_t* nan_count,
                      hipStream_t stream, const TableOut& tab = TableOut{}) {
  return launch_catalog_x3<DH, HB, VAR, 3>(d, indptr, indices, users, nb, region_of, coords,
                                           latlon_mat, scores, ld, nan_count, stream, tab);
}

template <int DH, int HB, int VAR>
int launch_forward(const DevParams& d, const int64_t* hist, int64_t b, int64_t n, int64_t hist_ld,
                   const int64_t* target, const int64_t* hreg, int64_t hreg_ld, const int64_t* treg,
                   const float* latlon, int64_t ll_ld, float* out, int32_t* nan_count, int32_t flags,
                   hipStream_t stream) {
  constexpr bool DIST = VarT<VAR>::DIST;
  const size_t lds = Consts<DH, HB, DIST>::BYTES;
  auto kern = forward_kernel<DH, HB, VAR>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  dim3 grid((unsigned)((b + CAND_PER_BLOCK - 1) / CAND_PER_BLOCK));
  hipLaunchKernelGGL(kern, grid, dim3(THREADS), lds, stream, d, hist, b, n, hist_ld, target, hreg,
                     hreg_ld, treg, latlon, ll_ld, out, nan_count, flags);
  return check_launch("forward_kernel");
}

// (DH, HB, VAR) -> template instance
#define NAIS_DISPATCH(FN, DH_, HB_, VAR_, ...)                                   \
  do {                                                                            \
    switch (VAR_) {                                                               \
      case 0: NAIS_DISPATCH_DH(FN, DH_, HB_, 0, __VA_ARGS__); break;              \
      case 1: NAIS_DISPATCH_DH(FN, DH_, HB_, 1, __VA_ARGS__); break;              \
      case 2: NAIS_DISPATCH_DH(FN, DH_, HB_, 2, __VA_ARGS__); break;              \
      default: NAIS_DISPATCH_DH(FN, DH_, HB_, 3, __VA_ARGS__); break;             \
    }                                                                             \
  } while (0)
#define NAIS_DISPATCH_DH(FN, DH_, HB_, V, ...)                                   \
  switch (DH_) {                                                                  \
    case 4: NAIS_DISPATCH_HB(FN, 4, HB_, V, __VA_ARGS__); break;                  \
    case 8: NAIS_DISPATCH_HB(FN, 8, HB_, V, __VA_ARGS__); break;                  \
    case 16: NAIS_DISPATCH_HB(FN, 16, HB_, V, __VA_ARGS__); break;                \
    case 32: NAIS_DISPATCH_HB(FN, 32, HB_, V, __VA_ARGS__); break;                \
    default: NAIS_DISPATCH_HB(FN, 64, HB_, V, __VA_ARGS__); break;                \
  }
#define NAIS_DISPATCH_HB(FN, DH, HB_, V, ...)                                    \
  switch (HB_) {                                                                  \
    case 1: rc = FN<DH, 1, V>(__VA_ARGS__); break;                                \
    case 2: rc = FN<DH, 2, V>(__VA_ARGS__); break;                                \
    case 4: rc = FN<DH, 4, V>(__VA_ARGS__); break;                                \
    default: rc = FN<DH, 8, V>(__VA_ARGS__); break;                               \
  }

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Every pr_d(d) = a * max(0.01, d)^b is finite and >= +0 for d in powerLaw.dist's range
// [0, pi * 6371] (a NaN distance takes the 0.01 branch): a > 0 and both ends finite (pr_d is
// monotone in d). Then a G product at +0.0 stays +0.0. The host-side twin for the pairs route is
// catalog._prior_entries_finite.
bool prior_zero_exit(double a, double b) {
  if (!std::isfinite(a) || !std::isfinite(b) || !(a > 0.0)) return false;
  const double lo = a * std::pow(0.01, b), hi = a * std::pow(3.141592653589793 * 6371.0, b);
  return std::isfinite(lo) && std::isfinite(hi);
}

int launch_prior(const double* coords, int64_t P, const int64_t* indptr, const int64_t* indices,
                 const int32_t* users, int nb, double a, double b, double* G, int64_t ld,
                 unsigned long long* gmax, hipStream_t st) {
  hipError_t e = hipMemsetAsync(gmax, 0, sizeof(unsigned long long) * nb, st);
  if (e != hipSuccess) return fail(NAIS_E_HIP, std::string("memset: ") + hipGetErrorString(e));
  dim3 grid((unsigned)((P + PRIOR_THREADS - 1) / PRIOR_THREADS), (unsigned)nb);
  hipLaunchKernelGGL(prior_kernel, grid, dim3(PRIOR_THREADS), 0, st, coords, P, indptr, indices,
                     users, a, b, G, ld, gmax, prior_zero_exit(a, b) ? 1 : 0);
  return check_launch("prior_kernel");
}

}  // namespace

int nais_internal_fail(int code, const char* msg) { return fail(code, msg); }
int nais_internal_stream_cus(hipStream_t stream) {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    return -1;
  uint32_t mask[32] = {};
  const uint32_t words = (uint32_t)std::min(32, (ncu + 31) / 32);
  if (hipExtStreamGetCUMask(stream, words, mask) != hipSuccess) return ncu;
  int n = 0;
  for (uint32_t i = 0; i < words; ++i) n += __builtin_popcount(mask[i]);
  return n > 0 ? std::min(n, ncu) : ncu;
}
int nais_internal_check_launch(const char* what) { return check_launch(what); }

extern "C" {

int32_t nais_abi_version(void) { return NAIS_ABI_VERSION; }

const char* nais_last_error(void) { return g_err.c_str(); }

int32_t nais_forward(const nais_params_t* params, const int64_t* hist, int64_t b, int64_t n,
                     int64_t hist_ld, const int64_t* target, const int64_t* hist_region,
                     int64_t hist_region_ld, const int64_t* target_region,
                     const float* target_lat_long, int64_t latlon_ld, float* out,
                     int32_t* nan_count, int32_t flags, void* stream) {
  Shape sh;
  int rc = validate(params, &sh);
  if (rc) return rc;
  if (b < 0 || n < 0) return fail(NAIS_E_INVALID, "negative b or n");
  if (b == 0) return NAIS_OK;
  if (!target || !out || (n > 0 && !hist)) return fail(NAIS_E_INVALID, "missing hist/target/out");
  const bool region = params->variant == NAIS_VARIANT_REGION ||
                      params->variant == NAIS_VARIANT_REGION_DISTANCE;
  const bool dist = params->variant == NAIS_VARIANT_REGION_DISTANCE ||
                    params->variant == NAIS_VARIANT_DISTANCE;
  if (region && (!target_region || (n > 0 && !hist_region)))
    return fail(NAIS_E_INVALID, "region variants need hist_region and target_region");
  if (dist && n > 0 && !target_lat_long)
    return fail(NAIS_E_INVALID, "region_distance needs target_lat_long");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  DevParams d;
  rc = to_dev(params, &d);
  if (rc) return rc;
  if (sh.gen_fwd)
    return nais_gx_forward(params, hist, b, n, hist_ld, target, hist_region, hist_region_ld,
                           target_region, target_lat_long, latlon_ld, out, nan_count, flags, st);
  NAIS_DISPATCH(launch_forward, sh.DH, sh.HB, params->variant, d, hist, b, n, hist_ld, target,
                hist_region, hist_region_ld, target_region, target_lat_long, latlon_ld, out,
                nan_count, flags, st);
  return rc;
}

size_t nais_score_topk_workspace_size(const nais_params_t* params, int32_t num_users, int32_t k,
                                      int32_t with_prior) {
  (void)k;
  if (!params || num_users <= 0) return 0;
  const int64_t nb = std::min<int64_t>(num_users, MAX_BATCH_USERS);
  const int64_t ld = round_up(params->num_pois, 64);
  size_t bytes = (size_t)(nb * ld * (int64_t)sizeof(float));
  if (with_prior) bytes += (size_t)(nb * ld * 8 + round_up(nb, 64) * 8);
  return bytes;
}

int32_t nais_score_topk(const nais_params_t* params, const int64_t* indptr, const int64_t* indices,
                        const int32_t* users, int32_t num_users, int32_t k,
                        const int64_t* region_of, const double* coords,
                        const double* latlon_mat, const nais_prior_t* prior,
                        int32_t* out_ids, float* out_scores, int32_t* nan_count,
                        int32_t* short_count, void* workspace, size_t workspace_bytes,
                        void* stream) {
  Shape sh;
  int rc = validate(params, &sh);
  if (rc) return rc;
  if (num_users < 0) return fail(NAIS_E_INVALID, "num_users < 0");
  if (num_users == 0) return NAIS_OK;
  if (k <= 0 || k > MAX_K) return fail(NAIS_E_UNSUPPORTED, "k must be in [1, 1024]");
  if (!indptr || !indices || !users || !out_ids || !out_scores)
    return fail(NAIS_E_INVALID, "missing indptr/indices/users/outputs");
  if ((params->variant == NAIS_VARIANT_REGION || params->variant == NAIS_VARIANT_REGION_DISTANCE) &&
      !region_of)
    return fail(NAIS_E_INVALID, "region variants need region_of");
  if ((params->variant == NAIS_VARIANT_REGION_DISTANCE || params->variant == NAIS_VARIANT_DISTANCE) &&
      !coords && !latlon_mat)
    return fail(NAIS_E_INVALID, "region_distance needs coords or latlon_mat");
  if (prior && !prior->coords) return fail(NAIS_E_INVALID, "prior needs coords");
  const size_t need = nais_score_topk_workspace_size(params, num_users, k, prior != nullptr);
  if (!workspace || workspace_bytes < need) return fail(NAIS_E_WORKSPACE, "workspace too small");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  DevParams d;
  rc = to_dev(params, &d);
  if (rc) return rc;
  float* scores = reinterpret_cast<float*>(workspace);
  const int64_t ld = round_up(params->num_pois, 64);
  for (int32_t u0 = 0; u0 < num_users; u0 += MAX_BATCH_USERS) {
    const int nb = std::min<int32_t>(MAX_BATCH_USERS, num_users - u0);
    if (sh.gen_cat)
      rc = nais_gx_catalog(params, indptr, indices, users + u0, nb, nullptr, 0, 0, 0, region_of,
                           coords, latlon_mat, scores, ld, nan_count, nullptr, nullptr, 0, st);
    else if (params->precision == NAIS_PRECISION_FP16X6)
      NAIS_DISPATCH(launch_catalog_x6b, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores, ld, nan_count, st);
    else if (params->precision == NAIS_PRECISION_FP16X6_PAIRSPLIT)
      NAIS_DISPATCH(launch_catalog_x6, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores, ld, nan_count, st);
    else if (params->precision == NAIS_PRECISION_FP16X3)
      NAIS_DISPATCH(launch_catalog_x3b, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores, ld, nan_count, st);
    else if (params->precision == NAIS_PRECISION_FP16X3_PAIRSPLIT)
      NAIS_DISPATCH(launch_catalog_x3, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores, ld, nan_count, st);
    else
      NAIS_DISPATCH(launch_catalog, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0, nb,
                    region_of, coords, latlon_mat, scores, ld, nan_count, st);
    if (rc) return rc;
    if (!prior) {
      hipLaunchKernelGGL(topk_kernel, dim3(nb), dim3(TOPK_THREADS), 0, st, scores, ld,
                         params->num_pois, k, out_ids + (int64_t)u0 * k,
                         out_scores + (int64_t)u0 * k, short_count);
      rc = check_launch("topk_kernel");
      if (rc) return rc;
    } else {
      const int64_t nbmax = std::min<int64_t>(num_users, MAX_BATCH_USERS);
      double* G = reinterpret_cast<double*>(scores + nbmax * ld);
      unsigned long long* gmax = reinterpret_cast<unsigned long long*>(G + nbmax * ld);
      rc = launch_prior(prior->coords, params->num_pois, indptr, indices, users + u0, nb, prior->a,
                        prior->b, G, ld, gmax, st);
      if (rc) return rc;
      hipLaunchKernelGGL(topk_blend_kernel, dim3(nb), dim3(TOPK_THREADS), 0, st, scores, ld, G, ld,
                         gmax, params->num_pois, k, (float)(1.0 - prior->alpha), prior->alpha,
                         out_ids + (int64_t)u0 * k, out_scores + (int64_t)u0 * k, short_count,
                         (double*)nullptr);
      rc = check_launch("topk_blend_kernel");
      if (rc) return rc;
    }
  }
  return NAIS_OK;
}

namespace {
// nais_pair_table: two row-major tables (e, es) with row pitch ld
int32_t pair_table_impl(const nais_params_t* params, const int64_t* items, int64_t num_items,
                        int64_t col0, int64_t cols, const int64_t* region_of, const double* coords,
                        const double* latlon_mat, float* e, float* es, int64_t ld, int32_t* work,
                        void* stream, bool split = false) {
  Shape sh;
  int rc = validate(params, &sh);
  if (rc) return rc;
  if (num_items < 0 || col0 < 0 || cols < 0 || col0 + cols > params->num_pois)
    return fail(NAIS_E_INVALID, "bad item count or column range");
  if (num_items == 0 || cols == 0) return NAIS_OK;
  if (!items || !e || !es) return fail(NAIS_E_INVALID, "missing pointer");
  if (ld < cols) return fail(NAIS_E_INVALID, "ld < cols");
  if ((params->variant == NAIS_VARIANT_REGION || params->variant == NAIS_VARIANT_REGION_DISTANCE) &&
      !region_of)
    return fail(NAIS_E_INVALID, "region variants need region_of");
  if ((params->variant == NAIS_VARIANT_REGION_DISTANCE || params->variant == NAIS_VARIANT_DISTANCE) &&
      !coords && !latlon_mat)
    return fail(NAIS_E_INVALID, "distance variants need coords or latlon_mat");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  DevParams d;
  rc = to_dev(params, &d);
  if (rc) return rc;
  if (sh.gen_tab)
    return nais_gx_catalog(params, nullptr, nullptr, nullptr, 0, items, num_items, col0, cols,
                           region_of, coords, latlon_mat, nullptr, 0, nullptr, e, es, ld, st, split);
  TableOut tab;
  if (split) {
    tab.sel_e = NAIS_SEL_HI;
    tab.ex = 1;
  }
  tab.ld = ld;
  tab.cols = cols;
  tab.gi = PAIR_GROUP_ITEMS;
  tab.work = work;
  const int64_t groups_per_launch = 65535;
  for (int64_t g0 = 0; g0 * tab.gi < num_items; g0 += groups_per_launch) {
    const int64_t base = g0 * tab.gi;
    tab.nitems = std::min<int64_t>(num_items - base, groups_per_launch * tab.gi);
    tab.e = e + base * ld;
    tab.es = es + base * ld * (split ? 2 : 1);
    tab.col0 = col0;
    const int ng = (int)((tab.nitems + tab.gi - 1) / tab.gi);
    if (params->precision == NAIS_PRECISION_FP32)
      NAIS_DISPATCH(launch_catalog, sh.DH, sh.HB, params->variant, d, nullptr, items + base, nullptr,
                    ng, region_of, coords, latlon_mat, nullptr, 0, nullptr, st, tab);
    else if (params->precision == NAIS_PRECISION_FP16X6 ||
             params->precision == NAIS_PRECISION_FP16X6_PAIRSPLIT)
      NAIS_DISPATCH(launch_catalog_x6b, sh.DH, sh.HB, params->variant, d, nullptr, items + base,
                    nullptr, ng, region_of, coords, latlon_mat, nullptr, 0, nullptr, st, tab);
    else
      NAIS_DISPATCH(launch_catalog_x3b, sh.DH, sh.HB, params->variant, d, nullptr, items + base,
                    nullptr, ng, region_of, coords, latlon_mat, nullptr, 0, nullptr, st, tab);
    if (rc) return rc;
  }
  return NAIS_OK;
}
}  // namespace

int32_t nais_pair_table(const nais_params_t* params, const int64_t* items, int64_t num_items,
                        int64_t col0, int64_t cols, const int64_t* region_of,
                        const double* coords, const double* latlon_mat, float* e, float* es,
                        int64_t ld, int32_t* work, void* stream) {
  return pair_table_impl(params, items, num_items, col0, cols, region_of, coords, latlon_mat, e, es,
                         ld, work, stream);
}

int32_t nais_pair_table_split(const nais_params_t* params, const int64_t* items, int64_t num_items,
                              int64_t col0, int64_t cols, const int64_t* region_of,
                              const double* coords, const double* latlon_mat, uint32_t* hi,
                              uint32_t* ex, int64_t ld, int32_t* work, void* stream) {
  return pair_table_impl(params, items, num_items, col0, cols, region_of, coords, latlon_mat,
                         reinterpret_cast<float*>(hi), reinterpret_cast<float*>(ex), ld, work, stream,
                         true);
}

int32_t nais_score_catalog(const nais_params_t* params, const int64_t* indptr,
                           const int64_t* indices, const int32_t* users, int32_t num_users,
                           const int64_t* region_of, const double* coords,
                           const double* latlon_mat, float* scores, int64_t score_ld,
                           int32_t* nan_count, void* stream) {
  Shape sh;
  int rc = validate(params, &sh);
  if (rc) return rc;
  if (num_users < 0) return fail(NAIS_E_INVALID, "num_users < 0");
  if (num_users == 0) return NAIS_OK;
  if (!indptr || !indices || !users || !scores) return fail(NAIS_E_INVALID, "missing pointer");
  if (score_ld < params->num_pois) return fail(NAIS_E_INVALID, "score_ld < num_pois");
  if ((params->variant == NAIS_VARIANT_REGION || params->variant == NAIS_VARIANT_REGION_DISTANCE) &&
      !region_of)
    return fail(NAIS_E_INVALID, "region variants need region_of");
  if ((params->variant == NAIS_VARIANT_REGION_DISTANCE || params->variant == NAIS_VARIANT_DISTANCE) &&
      !coords && !latlon_mat)
    return fail(NAIS_E_INVALID, "region_distance needs coords or latlon_mat");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  DevParams d;
  rc = to_dev(params, &d);
  if (rc) return rc;
  for (int32_t u0 = 0; u0 < num_users; u0 += 65535) {
    const int nb = std::min<int32_t>(65535, num_users - u0);
    if (sh.gen_cat)
      rc = nais_gx_catalog(params, indptr, indices, users + u0, nb, nullptr, 0, 0, 0, region_of,
                           coords, latlon_mat, scores + (int64_t)u0 * score_ld, score_ld, nan_count,
                           nullptr, nullptr, 0, st);
    else if (params->precision == NAIS_PRECISION_FP16X6)
      NAIS_DISPATCH(launch_catalog_x6b, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores + (int64_t)u0 * score_ld, score_ld,
                    nan_count, st);
    else if (params->precision == NAIS_PRECISION_FP16X6_PAIRSPLIT)
      NAIS_DISPATCH(launch_catalog_x6, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores + (int64_t)u0 * score_ld, score_ld,
                    nan_count, st);
    else if (params->precision == NAIS_PRECISION_FP16X3)
      NAIS_DISPATCH(launch_catalog_x3b, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores + (int64_t)u0 * score_ld, score_ld,
                    nan_count, st);
    else if (params->precision == NAIS_PRECISION_FP16X3_PAIRSPLIT)
      NAIS_DISPATCH(launch_catalog_x3, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0,
                    nb, region_of, coords, latlon_mat, scores + (int64_t)u0 * score_ld, score_ld,
                    nan_count, st);
    else
      NAIS_DISPATCH(launch_catalog, sh.DH, sh.HB, params->variant, d, indptr, indices, users + u0, nb,
                    region_of, coords, latlon_mat, scores + (int64_t)u0 * score_ld, score_ld,
                    nan_count, st);
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_topk_rows(const float* scores, int64_t score_ld, int64_t num_pois, int32_t num_rows,
                       int32_t k, int32_t* out_ids, float* out_scores, int32_t* short_count,
                       void* stream) {
  if (!scores || !out_ids || !out_scores || num_rows < 0 || num_pois <= 0 || score_ld < num_pois)
    return fail(NAIS_E_INVALID, "bad topk_rows arguments");
  if (k <= 0 || k > MAX_K) return fail(NAIS_E_UNSUPPORTED, "k must be in [1, 1024]");
  if (num_pois > 0xFFFFFFFFll) return fail(NAIS_E_UNSUPPORTED, "num_pois must fit 32 bits");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int32_t r0 = 0; r0 < num_rows; r0 += 65535) {
    const int nb = std::min<int32_t>(65535, num_rows - r0);
    hipLaunchKernelGGL(topk_kernel, dim3(nb), dim3(TOPK_THREADS), 0, st, scores + (int64_t)r0 * score_ld,
                       score_ld, num_pois, k, out_ids + (int64_t)r0 * k, out_scores + (int64_t)r0 * k,
                       short_count);
    const int rc = check_launch("topk_kernel");
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_powerlaw_prior(const double* coords, int64_t num_pois, const int64_t* indptr,
                            const int64_t* indices, const int32_t* users, int32_t num_users, double a,
                            double b, double* out, int64_t out_ld, double* out_max, void* stream) {
  if (!coords || !indptr || !indices || !users || !out || !out_max || num_pois <= 0 ||
      num_users < 0 || out_ld < num_pois)
    return fail(NAIS_E_INVALID, "bad powerlaw_prior arguments");
  if (num_pois > 65535ll * 256) return fail(NAIS_E_UNSUPPORTED, "num_pois too large");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int32_t u0 = 0; u0 < num_users; u0 += 65535) {
    const int nb = std::min<int32_t>(65535, num_users - u0);
    const int rc = launch_prior(coords, num_pois, indptr, indices, users + u0, nb, a, b,
                                out + (int64_t)u0 * out_ld, out_ld,
                                reinterpret_cast<unsigned long long*>(out_max + u0), st);
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_topk_blend_rows(const float* scores, int64_t score_ld, const double* g, int64_t g_ld,
                             const uint64_t* gmax_bits, int64_t num_pois, int32_t num_rows, int32_t k,
                             double alpha, int32_t* out_ids, float* out_scores, int32_t* short_count,
                             void* stream) {
  return nais_topk_blend_rows_f64(scores, score_ld, g, g_ld, gmax_bits, num_pois, num_rows, k, alpha,
                                  out_ids, out_scores, nullptr, short_count, stream);
}

int32_t nais_topk_merge_f64(const double* keys, const int64_t* ids, int32_t num_rows, int32_t m,
                            int32_t k, int64_t* out_ids, float* out_scores, double* out_keys,
                            void* stream) {
  if (num_rows < 0 || m <= 0 || k <= 0 || k > m) return fail(NAIS_E_INVALID, "bad shape");
  if (m > MERGE_CAP) return fail(NAIS_E_UNSUPPORTED, "m > 2048 candidates per row");
  if (num_rows == 0) return NAIS_OK;
  if (!keys || !ids || !out_ids || !out_scores) return fail(NAIS_E_INVALID, "missing pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int32_t r0 = 0; r0 < num_rows; r0 += 65535) {
    const int nb = std::min<int32_t>(65535, num_rows - r0);
    hipLaunchKernelGGL(topk_merge_f64_kernel, dim3(nb), dim3(MERGE_THREADS), 0, st,
                       keys + (int64_t)r0 * m, ids + (int64_t)r0 * m, (int)m, (int)k,
                       out_ids + (int64_t)r0 * k, out_scores + (int64_t)r0 * k,
                       out_keys ? out_keys + (int64_t)r0 * k : nullptr);
    const int rc = check_launch("topk_merge_f64_kernel");
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_topk_blend_rows_f64(const float* scores, int64_t score_ld, const double* g, int64_t g_ld,
                                 const uint64_t* gmax_bits, int64_t num_pois, int32_t num_rows, int32_t k,
                                 double alpha, int32_t* out_ids, float* out_scores, double* out_blend,
                                 int32_t* short_count, void* stream) {
  if (num_rows < 0 || num_pois <= 0 || k <= 0 || score_ld < num_pois || g_ld < num_pois)
    return fail(NAIS_E_INVALID, "bad shape");
  if (k > MAX_K) return fail(NAIS_E_UNSUPPORTED, "k > 1024");
  if (num_rows == 0) return NAIS_OK;
  if (!scores || !g || !gmax_bits || !out_ids || !out_scores) return fail(NAIS_E_INVALID, "missing pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int32_t r0 = 0; r0 < num_rows; r0 += 65535) {
    const int nb = std::min<int32_t>(65535, num_rows - r0);
    hipLaunchKernelGGL(topk_blend_kernel, dim3(nb), dim3(TOPK_THREADS), 0, st, scores + (int64_t)r0 * score_ld,
                       score_ld, g + (int64_t)r0 * g_ld, g_ld,
                       reinterpret_cast<const unsigned long long*>(gmax_bits) + r0, num_pois, k,
                       (float)(1.0 - alpha), alpha, out_ids + (int64_t)r0 * k, out_scores + (int64_t)r0 * k,
                       short_count, out_blend ? out_blend + (int64_t)r0 * k : nullptr);
    const int rc = check_launch("topk_blend_kernel");
    if (rc) return rc;
  }
  return NAIS_OK;
}

int32_t nais_distance_histogram(const double* coords, const int64_t* indptr, const int64_t* indices,
                                int64_t num_users, uint64_t* hist, int64_t nbins, uint64_t* overflow,
                                void* stream) {
  if (!coords || !indptr || !indices || !hist || !overflow || num_users < 0 || nbins <= 0)
    return fail(NAIS_E_INVALID, "bad distance_histogram arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(hist, 0, sizeof(uint64_t) * nbins, st);
  if (e == hipSuccess) e = hipMemsetAsync(overflow, 0, sizeof(uint64_t), st);
  if (e != hipSuccess) return fail(NAIS_E_HIP, std::string("memset: ") + hipGetErrorString(e));
  if (num_users == 0) return NAIS_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>(num_users, 4096);
  hipLaunchKernelGGL(distance_histogram_kernel, dim3(blocks), dim3(256), 0, st, coords, indptr, indices,
                     num_users, reinterpret_cast<unsigned long long*>(hist), nbins,
                     reinterpret_cast<unsigned long long*>(overflow));
  return check_launch("distance_histogram_kernel");
}

int32_t nais_gather_rows(const float* table, int64_t rows, int32_t dim, const int64_t* idx,
                         int64_t m, float* out, void* stream) {
  if (!table || !idx || !out || rows <= 0 || dim <= 0 || m < 0)
    return fail(NAIS_E_INVALID, "bad gather arguments");
  if (m == 0) return NAIS_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool vec = dim % 4 == 0 && (reinterpret_cast<uintptr_t>(table) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  const int64_t total = vec ? m * (dim / 4) : m * dim;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 16);
  if (vec)
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                       reinterpret_cast<const nf4*>(table), dim / 4, idx, m,
                       reinterpret_cast<nf4*>(out));
  else
    hipLaunchKernelGGL(gather_rows_scalar_kernel, dim3((unsigned)blocks), dim3(256), 0, st, table,
                       dim, idx, m, out);
  return check_launch("gather_rows_kernel");
}

}  // extern "C"
