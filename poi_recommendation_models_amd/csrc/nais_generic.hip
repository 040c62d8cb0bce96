// nais_generic.hip -- the scoring entry points at the shapes the tuned kernels are not compiled
// for: embed widths other than 8 / 16 / 32 / 64 / 128 up to GX_MAX_D = 256, hidden sizes above
// 256 (any), and hidden > 128 at the precisions whose catalog kernels stop there. The reference
// builds Linear(embed_size, hidden_size) for any sizes (model.py:9-38, 100-130, 190-229); these
// kernels make the C-ABI take them as they are, in exact fp32 (nais_gx.h: one hidden block of W1
// at a time in LDS, 32 history items x one target per MFMA tile, two targets per wave).
//
//   gx_catalog_kernel  per-user catalog rows (nais_score_catalog / nais_score_topk): one workgroup
//                      per (user, 32-candidate tile), the user's history in 32-item chunks, S / N
//                      accumulated over the chunks; history POIs scored -1 (batches.py:56). Also the
//                      pair-table mode (nais_pair_table): (32-item group, 32-candidate tile) ->
//                      e = exp(a) [item != c] and e (h . t) per pair.
//   gx_forward_kernel  nais_forward: per-row histories (one row per wave, its items staged in the
//                      wave's own LDS rows) or a history shared by every row (hist_ld == 0:
//                      32 rows per workgroup over one staged chunk).
// Semantics as the tuned kernels: mask model.py:92-95, exp without max-subtraction model.py:75,
// (sum e)^beta model.py:80-82, NaN counting model.py:50-54, sigmoid model.py:55.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <cmath>

#include "nais.h"
#include "nais_gx.h"
#include "nais_internal.h"

namespace {

using gx::GX_NT;
using gx::GX_TT;
using gx::Shape;

struct GxP {
  const float *eh, *et, *er, *w1, *b1, *w2, *wd, *bd;
  int64_t P;
  int D, IDIM, RDIM, H, DIN;   // D = IDIM + RDIM: the full [item | region] row
  float beta, dscale;
};

GxP gx_params(const nais_params_t* p) {
  GxP g;
  g.eh = p->embed_history;
  g.et = p->embed_target;
  g.er = p->embed_region;
  g.w1 = p->w1;
  g.b1 = p->b1;
  g.w2 = p->w2;
  g.wd = p->dist_w;
  g.bd = p->dist_b;
  g.P = p->num_pois;
  g.D = p->embed_dim;
  const bool region = p->variant == NAIS_VARIANT_REGION || p->variant == NAIS_VARIANT_REGION_DISTANCE;
  g.IDIM = region ? p->item_dim : p->embed_dim;
  g.RDIM = region ? p->region_dim : 0;
  g.H = p->hidden;
  g.DIN = p->din;
  g.beta = p->beta;
  g.dscale = p->variant == NAIS_VARIANT_DISTANCE ? 1000.f : 100.f;   // model.py:369 / :265
  return g;
}

// element d of the full row of POI `item` (region id `reg`): [table[item] | embed_region[reg]]
__device__ __forceinline__ float full_row(const GxP& p, const float* tab, int64_t item, int64_t reg, int d) {
  if (d < p.IDIM) return tab[item * p.IDIM + d];
  return p.er[reg * p.RDIM + (d - p.IDIM)];
}

__device__ __forceinline__ float finish_logit(float S, float N, float beta, bool empty) {
  if (empty) return 0.f;   // sum over an empty history dim (model.py:79-88 with n == 0)
  const float den = (beta == 0.5f) ? sqrtf(S) : powf(S, beta);
  return N / den;
}

constexpr int al4(int x) { return (x + 3) & ~3; }

// ---------------------------------------------------------------------------------------------
// Catalog rows / pair tables
// ---------------------------------------------------------------------------------------------
struct CatArgs {
  const int64_t* indptr;    // catalog: CSR of the users; table: nullptr
  const int64_t* indices;   // catalog: CSR indices; table: the item list
  const int32_t* users;
  const int64_t* region_of;
  const double* coords;
  const double* latlon_mat;
  float* scores;            // catalog: [slot][ld]
  int64_t score_ld;
  int32_t* nan_count;
  float* e;                 // table: e / es [row][ld] (e != nullptr selects the table mode)
  float* es;
  int64_t ld, col0, cols, nitems;
  uint32_t sel_e;           // the e words (float or the split16 hi, nais_internal.h)
  int32_t ex;               // split16: es holds (e, e*s) pairs, row pitch 2 * ld
};

struct CatLds {
  int o_w, o_bw, o_h, o_t, o_f, o_id, o_co, o_tc, total;   // float offsets
  __host__ __device__ CatLds(const Shape& s, bool dist) {
    o_w = 0;
    o_bw = al4(32 * s.Q);
    o_h = o_bw + 64;
    o_t = al4(o_h + 32 * s.HP);
    o_f = al4(o_t + GX_TT * s.D);
    o_id = al4(o_f + (dist ? GX_TT * 64 : 0));
    o_co = o_id + 64;                // 32 int64 item ids
    o_tc = o_co + (dist ? 128 : 0);  // 32 x 2 double item coords
    total = o_tc + (dist ? 128 : 0); // 32 x 2 double target coords
  }
};

template <bool DIST>
__global__ void __launch_bounds__(GX_NT, 1) gx_catalog_kernel(GxP p, CatArgs a) {
  extern __shared__ float4 gx_lds4[];
  float* L = reinterpret_cast<float*>(gx_lds4);
  const Shape s(p.D, p.DIN, p.H);
  const CatLds o(s, DIST);
  float *Lw = L + o.o_w, *Lbw = L + o.o_bw, *Lh = L + o.o_h, *Lt = L + o.o_t, *Lf = L + o.o_f;
  int64_t* Lid = reinterpret_cast<int64_t*>(L + o.o_id);
  double* Lco = reinterpret_cast<double*>(L + o.o_co);
  double* Ltc = reinterpret_cast<double*>(L + o.o_tc);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 31, hh = lane >> 5;
  const bool tab = a.e != nullptr;
  int64_t hbeg, hlen;
  if (tab) {
    hbeg = int64_t(blockIdx.y) * 32;
    hlen = std::min<int64_t>(32, a.nitems - hbeg);
  } else {
    const int64_t u = a.users[blockIdx.y];
    hbeg = a.indptr[u];
    hlen = a.indptr[u + 1] - hbeg;
  }
  const int64_t c0 = a.col0 + int64_t(blockIdx.x) * GX_TT;
  const int64_t cend = tab ? a.col0 + a.cols : p.P;
  for (int f = tid; f < GX_TT * s.D; f += GX_NT) {
    const int tq = f / s.D, d = f % s.D;
    const int64_t c = c0 + tq;
    Lt[f] = c < cend ? full_row(p, p.et, c, p.RDIM ? a.region_of[c] : 0, d) : 0.f;
  }
  if (DIST && a.coords && tid < GX_TT) {
    const int64_t c = std::min<int64_t>(c0 + tid, cend - 1);
    Ltc[2 * tid] = a.coords[2 * c];
    Ltc[2 * tid + 1] = a.coords[2 * c + 1];
  }
  float S[8], N[8];
  bool inh[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    S[t] = N[t] = 0.f;
    inh[t] = false;
  }
  for (int64_t j0 = 0; j0 < hlen; j0 += 32) {
    const int jn = (int)std::min<int64_t>(32, hlen - j0);
    __syncthreads();   // the previous chunk's readers are done
    for (int f = tid; f < 32 * s.D; f += GX_NT) {
      const int jj = f / s.D, d = f % s.D;
      float v = 0.f;
      if (jj < jn) {
        const int64_t item = a.indices[hbeg + j0 + jj];
        v = full_row(p, p.eh, item, p.RDIM ? a.region_of[item] : 0, d);
      }
      Lh[jj * s.HP + d] = v;
    }
    if (tid < 32) {
      const int64_t item = tid < jn ? a.indices[hbeg + j0 + tid] : -1;
      Lid[tid] = item;
      if (DIST && a.coords) {
        Lco[2 * tid] = item >= 0 ? a.coords[2 * item] : 0.0;
        Lco[2 * tid + 1] = item >= 0 ? a.coords[2 * item + 1] : 0.0;
      }
    }
    __syncthreads();
    if (DIST) {   // the pairs' 2 features (run.py:51-52 in float64, cast to float32; model.py:265)
      for (int f = tid; f < GX_TT * 32; f += GX_NT) {
        const int tq = f >> 5, jj = f & 31;
        const int64_t c = std::min<int64_t>(c0 + tq, cend - 1), item = Lid[jj];
        float l0 = 0.f, l1 = 0.f;
        if (item >= 0) {
          if (a.coords) {
            l0 = (float)fabs(Ltc[2 * tq] - Lco[2 * jj]);
            l1 = (float)fabs(Ltc[2 * tq + 1] - Lco[2 * jj + 1]);
          } else {
            const double* ll = a.latlon_mat + (c * p.P + item) * 2;
            l0 = (float)ll[0];
            l1 = (float)ll[1];
          }
        }
        Lf[2 * f] = gx::dist_feat(p.wd, p.bd, p.dscale, l0, l1, 0);
        Lf[2 * f + 1] = gx::dist_feat(p.wd, p.bd, p.dscale, l0, l1, 1);
      }
    }
    float pa[8], sd[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) pa[t] = sd[t] = 0.f;
    for (int hb = 0; hb < s.HB; ++hb) {
      if (hb > 0) __syncthreads();   // every wave is done with the previous block
      gx::stage_w1_block(p.w1, p.b1, p.w2, s, hb, Lw, Lbw, tid, GX_NT);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ta = w * 8 + 2 * q;
        gx::block_logits<true, DIST, false>(s, Lw, Lbw, Lh, Lt + ta * s.D, Lt + (ta + 1) * s.D,
                                            Lf + ta * 64, Lf + (ta + 1) * 64, lane, hb, hb == 0,
                                            pa[2 * q], pa[2 * q + 1], sd[2 * q], sd[2 * q + 1],
                                            gx::NoDrop{}, 0u, 0u);
      }
    }
    const int64_t item = Lid[n];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int64_t c = c0 + w * 8 + t;
      const float at = pa[t] + __shfl_xor(pa[t], 32), st = sd[t] + __shfl_xor(sd[t], 32);
      const bool valid = n < jn;
      const float e = valid ? expf(at) * (item != c ? 1.f : 0.f) : 0.f;   // model.py:75-78
      if (tab) {
        if (valid && hh == 0 && c < cend) {
          const int64_t o2 = (hbeg + n) * a.ld + (c - a.col0);
          const uint32_t eb = __float_as_uint(e), sb = __float_as_uint(e * st);
          a.e[o2] = __uint_as_float(__builtin_amdgcn_perm(sb, eb, a.sel_e));
          if (a.ex) reinterpret_cast<float2*>(a.es)[o2] = make_float2(e, e * st);
          else a.es[o2] = e * st;
        }
      } else {
        S[t] += gx::half_sum32(e);
        N[t] += gx::half_sum32(e * st);
        inh[t] |= __ballot(valid && item == c) != 0ull;
      }
    }
  }
  if (tab) return;
  int nans = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int64_t c = c0 + w * 8 + t;
    const float logit = finish_logit(S[t], N[t], p.beta, hlen == 0);
    const bool isnan_ = logit != logit;
    float sc = 1.0f / (1.0f + expf(-logit));
    if (isnan_) sc = __builtin_nanf("");
    if (inh[t]) sc = -1.f;   // history POI: not a candidate (batches.py:56)
    if (lane == t && c < cend) a.scores[int64_t(blockIdx.y) * a.score_ld + c] = sc;
    nans += (c < cend && !inh[t] && isnan_) ? 1 : 0;
  }
  if (a.nan_count && lane == 0 && nans) atomicAdd(a.nan_count, nans);
}

// ---------------------------------------------------------------------------------------------
// nais_forward
// ---------------------------------------------------------------------------------------------
struct FwdArgs {
  const int64_t* hist;
  int64_t b, n, hist_ld;
  const int64_t* target;
  const int64_t* hreg;
  int64_t hreg_ld;
  const int64_t* treg;
  const float* ll;
  int64_t ll_ld;
  float* out;
  int32_t* nan_count;
  int32_t flags;
};

// per-row histories: NW waves, one row each (its own h rows); shared history (hist_ld == 0 and
// hreg_ld == 0): 4 waves x 8 rows over one staged chunk
struct FwdLds {
  int o_w, o_bw, o_h, o_t, o_f, o_id, total;
  __host__ __device__ FwdLds(const Shape& s, bool dist, bool per_row, int nw) {
    const int hsets = per_row ? nw : 1, rows = per_row ? nw : GX_TT;
    o_w = 0;
    o_bw = al4(32 * s.Q);
    o_h = o_bw + 64;
    o_t = al4(o_h + hsets * 32 * s.HP);
    o_f = al4(o_t + rows * s.D);
    o_id = al4(o_f + (dist ? rows * 64 : 0));
    total = o_id + hsets * 64;
  }
};

template <bool DIST, bool PER_ROW>
__global__ void __launch_bounds__(GX_NT, 1) gx_forward_kernel(GxP p, FwdArgs a) {
  extern __shared__ float4 gx_lds4[];
  float* L = reinterpret_cast<float*>(gx_lds4);
  const Shape s(p.D, p.DIN, p.H);
  const int nw = blockDim.x >> 6;
  const FwdLds o(s, DIST, PER_ROW, nw);
  float *Lw = L + o.o_w, *Lbw = L + o.o_bw;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = lane & 31, hh = lane >> 5;
  const int nt = blockDim.x;
  constexpr int TPW = PER_ROW ? 1 : 8;          // rows per wave
  const int rows = PER_ROW ? nw : GX_TT;        // rows per workgroup
  const int64_t r0 = int64_t(blockIdx.x) * rows;
  float* Lt = L + o.o_t;
  float* Lf = L + o.o_f;
  for (int f = tid; f < rows * s.D; f += nt) {
    const int rq = f / s.D, d = f % s.D;
    const int64_t r = std::min<int64_t>(r0 + rq, a.b - 1);
    Lt[f] = full_row(p, p.et, a.target[r], p.RDIM ? a.treg[r] : 0, d);
  }
  float S[TPW], N[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) S[t] = N[t] = 0.f;
  for (int64_t j0 = 0; j0 < a.n; j0 += 32) {
    const int jn = (int)std::min<int64_t>(32, a.n - j0);
    __syncthreads();
    // h rows: per wave (its row's items) or once (the shared history)
    for (int f = tid; f < (PER_ROW ? nw : 1) * 32 * s.D; f += nt) {
      const int set = f / (32 * s.D), rem = f % (32 * s.D), jj = rem / s.D, d = rem % s.D;
      const int64_t r = std::min<int64_t>(r0 + set, a.b - 1);
      float v = 0.f;
      if (jj < jn) {
        const int64_t j = j0 + jj;
        v = full_row(p, p.eh, a.hist[r * a.hist_ld + j], p.RDIM ? a.hreg[r * a.hreg_ld + j] : 0, d);
      }
      L[o.o_h + set * 32 * s.HP + jj * s.HP + d] = v;
    }
    for (int f = tid; f < (PER_ROW ? nw : 1) * 32; f += nt) {
      const int set = f >> 5, jj = f & 31;
      const int64_t r = std::min<int64_t>(r0 + set, a.b - 1);
      reinterpret_cast<int64_t*>(L + o.o_id)[f] = jj < jn ? a.hist[r * a.hist_ld + j0 + jj] : -1;
    }
    if (DIST) {
      for (int f = tid; f < rows * 32; f += nt) {
        const int rq = f >> 5, jj = f & 31;
        const int64_t r = std::min<int64_t>(r0 + rq, a.b - 1);
        float l0 = 0.f, l1 = 0.f;
        if (jj < jn) {
          const float* ll = a.ll + r * a.ll_ld + 2 * (j0 + jj);
          l0 = ll[0];
          l1 = ll[1];
        }
        Lf[2 * f] = gx::dist_feat(p.wd, p.bd, p.dscale, l0, l1, 0);
        Lf[2 * f + 1] = gx::dist_feat(p.wd, p.bd, p.dscale, l0, l1, 1);
      }
    }
    float pa[TPW], sd[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) pa[t] = sd[t] = 0.f;
    const float* Lh = L + o.o_h + (PER_ROW ? w * 32 * s.HP : 0);
    for (int hb = 0; hb < s.HB; ++hb) {
      __syncthreads();
      gx::stage_w1_block(p.w1, p.b1, p.w2, s, hb, Lw, Lbw, tid, nt);
      __syncthreads();
      if (PER_ROW) {
        float dummy0 = 0.f, dummy1 = 0.f;
        gx::block_logits<false, DIST, false>(s, Lw, Lbw, Lh, Lt + w * s.D, Lt + w * s.D, Lf + w * 64,
                                             Lf + w * 64, lane, hb, hb == 0, pa[0], dummy0, sd[0],
                                             dummy1, gx::NoDrop{}, 0u, 0u);
      } else {
#pragma unroll
        for (int q = 0; q < TPW / 2; ++q) {
          const int ta = w * 8 + 2 * q;
          gx::block_logits<true, DIST, false>(s, Lw, Lbw, Lh, Lt + ta * s.D, Lt + (ta + 1) * s.D,
                                              Lf + ta * 64, Lf + (ta + 1) * 64, lane, hb, hb == 0,
                                              pa[2 * q], pa[2 * q + 1], sd[2 * q], sd[2 * q + 1],
                                              gx::NoDrop{}, 0u, 0u);
        }
      }
    }
    const int64_t item = reinterpret_cast<const int64_t*>(L + o.o_id)[(PER_ROW ? w * 32 : 0) + n];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int64_t r = std::min<int64_t>(r0 + (PER_ROW ? w : w * 8 + t), a.b - 1);
      const float at = pa[t] + __shfl_xor(pa[t], 32), st = sd[t] + __shfl_xor(sd[t], 32);
      const float e = n < jn ? expf(at) * (item != a.target[r] ? 1.f : 0.f) : 0.f;
      S[t] += gx::half_sum32(e);
      N[t] += gx::half_sum32(e * st);
    }
  }
  int nans = 0;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int64_t r = r0 + (PER_ROW ? w : w * 8 + t);
    const float logit = finish_logit(S[t], N[t], p.beta, a.n == 0);
    const bool isnan_ = logit != logit;
    const float v = (a.flags & NAIS_FLAG_SIGMOID) ? 1.0f / (1.0f + expf(-logit)) : logit;
    if (lane == t && r < a.b) a.out[r] = v;
    nans += (r < a.b && isnan_) ? 1 : 0;
  }
  if (a.nan_count && lane == 0 && nans) atomicAdd(a.nan_count, nans);
}

template <typename K>
void set_lds_once(K kern) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

constexpr size_t kLds = 160 * 1024;

int gx_check(const nais_params_t* p) {
  const int D = p->embed_dim;
  if (D < 1 || D > gx::GX_MAX_D)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "embed_dim above 256: the generic kernels hold a "
                                                  "256-wide h chunk and target tile in LDS");
  return NAIS_OK;
}

}  // namespace

int nais_gx_catalog(const nais_params_t* params, const int64_t* indptr, const int64_t* indices,
                    const int32_t* users, int nb, const int64_t* items, int64_t nitems, int64_t col0,
                    int64_t cols, const int64_t* region_of, const double* coords,
                    const double* latlon_mat, float* scores, int64_t score_ld, int32_t* nan_count,
                    float* e, float* es, int64_t ld, hipStream_t st, int split) {
  int rc = gx_check(params);
  if (rc) return rc;
  const GxP p = gx_params(params);
  const bool dist = params->variant == NAIS_VARIANT_REGION_DISTANCE ||
                    params->variant == NAIS_VARIANT_DISTANCE;
  const Shape s(p.D, p.DIN, p.H);
  const size_t lds = size_t(CatLds(s, dist).total) * 4;
  if (lds > kLds) return nais_internal_fail(NAIS_E_UNSUPPORTED, "generic catalog kernel: LDS budget");
  static bool once = (set_lds_once(gx_catalog_kernel<false>), set_lds_once(gx_catalog_kernel<true>), true);
  (void)once;
  CatArgs a{};
  a.indptr = indptr;
  a.users = users;
  a.region_of = region_of;
  a.coords = coords;
  a.latlon_mat = latlon_mat;
  a.scores = scores;
  a.score_ld = score_ld;
  a.nan_count = nan_count;
  a.sel_e = split ? NAIS_SEL_HI : NAIS_SEL_E;
  a.ex = split ? 1 : 0;
  auto kern = dist ? gx_catalog_kernel<true> : gx_catalog_kernel<false>;
  if (!e) {   // catalog rows: grid (candidate tiles, users)
    a.indices = indices;
    a.col0 = 0;
    dim3 grid((unsigned)((p.P + GX_TT - 1) / GX_TT), (unsigned)nb);
    hipLaunchKernelGGL(kern, grid, dim3(GX_NT), lds, st, p, a);
    return nais_internal_check_launch("gx_catalog_kernel");
  }
  a.e = e;   // pair tables: grid (candidate tiles, 32-item groups), 65535 groups per launch
  a.es = es;
  a.ld = ld;
  a.col0 = col0;
  a.cols = cols;
  for (int64_t base = 0; base < nitems; base += int64_t(65535) * 32) {
    a.indices = items + base;
    a.nitems = std::min<int64_t>(nitems - base, int64_t(65535) * 32);
    a.e = e + base * ld;
    a.es = es + base * ld * (split ? 2 : 1);
    dim3 grid((unsigned)((cols + GX_TT - 1) / GX_TT), (unsigned)((a.nitems + 31) / 32));
    hipLaunchKernelGGL(kern, grid, dim3(GX_NT), lds, st, p, a);
    if ((rc = nais_internal_check_launch("gx_catalog_kernel (table)"))) return rc;
  }
  return NAIS_OK;
}

int nais_gx_forward(const nais_params_t* params, const int64_t* hist, int64_t b, int64_t n,
                    int64_t hist_ld, const int64_t* target, const int64_t* hreg, int64_t hreg_ld,
                    const int64_t* treg, const float* latlon, int64_t ll_ld, float* out,
                    int32_t* nan_count, int32_t flags, hipStream_t st) {
  int rc = gx_check(params);
  if (rc) return rc;
  const GxP p = gx_params(params);
  const bool dist = params->variant == NAIS_VARIANT_REGION_DISTANCE ||
                    params->variant == NAIS_VARIANT_DISTANCE;
  const bool region = p.RDIM > 0;
  const bool per_row = hist_ld != 0 || (region && hreg_ld != 0);
  const Shape s(p.D, p.DIN, p.H);
  int nw = 4;
  if (per_row && size_t(FwdLds(s, dist, true, 4).total) * 4 > kLds) nw = 2;
  const size_t lds = size_t(FwdLds(s, dist, per_row, nw).total) * 4;
  if (lds > kLds) return nais_internal_fail(NAIS_E_UNSUPPORTED, "generic forward kernel: LDS budget");
  static bool once = (set_lds_once(gx_forward_kernel<false, false>), set_lds_once(gx_forward_kernel<false, true>),
                      set_lds_once(gx_forward_kernel<true, false>), set_lds_once(gx_forward_kernel<true, true>), true);
  (void)once;
  FwdArgs a{hist, b, n, hist_ld, target, hreg, hreg_ld, treg, latlon, ll_ld, out, nan_count, flags};
  const int rows = per_row ? nw : GX_TT;
  dim3 grid((unsigned)((b + rows - 1) / rows));
  auto kern = dist ? (per_row ? gx_forward_kernel<true, true> : gx_forward_kernel<true, false>)
                   : (per_row ? gx_forward_kernel<false, true> : gx_forward_kernel<false, false>);
  hipLaunchKernelGGL(kern, grid, dim3(per_row ? nw * 64 : GX_NT), lds, st, p, a);
  return nais_internal_check_launch("gx_forward_kernel");
}
