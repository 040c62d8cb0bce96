// nais_dot.hip -- transform_attn's dot-product attention core (model.py:1959-2098).
//
// transform_attn pools near-POI context like New4 (rows xh = [E_hist | in | out], xt =
// [E_tgt | out | in]) but replaces the NAIS MLP with projections of the full rows
// (model.py:2030-2033):  q = query(t_c), k_j = key(h_j), v_j = value(h_j),
//   logit_j = sum(q * k_j) / sqrt(E);  prediction = sum_j m_j e_j (v_j . t_c) / (sum_j m_j e_j)^beta
// with e_j = exp(logit_j) and the usual mask m_j = [h_j != c]. q, k, v depend on one POI each, so
// the projections become three per-POI tables (nais_linear_rows): qt = xt Wq^T + bq,
// kh = xh Wk^T + bk, vh = xh Wv^T + bv, and a (history item j, candidate c) term needs only two
// D-dots: e_jc = exp(qt_c . kh_j / sqrt(E)), s_jc = vh_j . xt_c.
//
// One-item histories: result2 is already [b, n], so exp_A.squeeze(dim=-1) (model.py:2042) makes
// it [b] for n == 1 and `exp_A * mask` broadcasts to [b, b]: every row then pools exp over ALL b
// rows of the call, pred_r = m_r s_r S / (m_r S)^beta, S = sum_r' e_r'. nais_dot_forward restates
// that for n == 1 calls; nais_dot_single_fixup restates it for new4_validation's 1024-candidate
// chunks (validation.py:262-270) of users with one history item.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "nais.h"
#include "nais_internal.h"

namespace {

// ------------------------------------------------------------------ y = x W^T + b over rows
// 256 threads; W^T staged in LDS as [din][dout] (conflict-free along outputs); each thread owns
// one (row, output) per pass.
__global__ void __launch_bounds__(256)
linear_rows_kernel(const float* __restrict__ x, int64_t x_ld, int64_t rows, int din,
                   const float* __restrict__ w, const float* __restrict__ b, int dout,
                   float* __restrict__ y, int64_t y_ld) {
  extern __shared__ float wt[];   // [din][dout]
  for (int f = threadIdx.x; f < din * dout; f += 256) {
    const int o = f / din, i = f % din;
    wt[i * dout + o] = w[f];
  }
  __syncthreads();
  const int rows_per = 256 / dout;                 // dout <= 256
  const int o = threadIdx.x % dout, rl = threadIdx.x / dout;
  if (rl >= rows_per) return;
  const float bo = b ? b[o] : 0.f;
  for (int64_t r = int64_t(blockIdx.x) * rows_per + rl; r < rows; r += int64_t(gridDim.x) * rows_per) {
    const float* xr = x + r * x_ld;
    float acc = 0.f;
    for (int i = 0; i < din; ++i) acc = fmaf(xr[i], wt[i * dout + o], acc);
    y[r * y_ld + o] = acc + bo;
  }
}

struct Tabs {
  int D;
  float beta, scale;           // logit = dot / scale (torch's true division, model.py:2033)
  const float *xh, *xt, *qt, *kh, *vh;
};

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// ------------------------------------------------------------------ forward, n >= 2 (or 0)
// one wave per row; lanes over D (D <= 128 -> 2 elements per lane at most)
constexpr int FW = 4;
__global__ void __launch_bounds__(FW * 64)
dot_forward_kernel(Tabs t, const int64_t* __restrict__ hist, int64_t b, int64_t n, int64_t hist_ld,
                   const int64_t* __restrict__ target, float* __restrict__ out, int sigmoid,
                   int32_t* __restrict__ nan_count) {
  const int lane = threadIdx.x & 63;
  const int64_t r = int64_t(blockIdx.x) * FW + (threadIdx.x >> 6);
  if (r >= b) return;
  const int64_t c = target[r];
  const int D = t.D;
  float q0 = 0.f, q1 = 0.f, x0 = 0.f, x1 = 0.f;
  if (lane < D) { q0 = t.qt[c * D + lane]; x0 = t.xt[c * D + lane]; }
  if (lane + 64 < D) { q1 = t.qt[c * D + lane + 64]; x1 = t.xt[c * D + lane + 64]; }
  float S = 0.f, N = 0.f;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t h = hist[r * hist_ld + j];
    float k0 = 0.f, k1 = 0.f, v0 = 0.f, v1 = 0.f;
    if (lane < D) { k0 = t.kh[h * D + lane]; v0 = t.vh[h * D + lane]; }
    if (lane + 64 < D) { k1 = t.kh[h * D + lane + 64]; v1 = t.vh[h * D + lane + 64]; }
    const float l = wave_sum(fmaf(q1, k1, q0 * k0)) / t.scale;
    const float s = wave_sum(fmaf(v1, x1, v0 * x0));
    const float e = (h != c) ? expf(l) : 0.f;
    S += e;
    N = fmaf(e, s, N);
  }
  float logit = (n > 0) ? N / ((t.beta == 0.5f) ? sqrtf(S) : powf(S, t.beta)) : 0.f;
  if (lane == 0) {
    out[r] = sigmoid ? sigm(logit) : logit;
    if (nan_count && logit != logit) atomicAdd(nan_count, 1);
  }
}

// ------------------------------------------------------------------ forward, n == 1 (batch-coupled)
// one workgroup of 1024 threads: pass 1 S = sum_r exp(logit_r) (unmasked), pass 2 the outputs
__global__ void __launch_bounds__(1024)
dot_forward_single_kernel(Tabs t, const int64_t* __restrict__ hist, int64_t b, int64_t hist_ld,
                          const int64_t* __restrict__ target, float* __restrict__ out, int sigmoid,
                          int32_t* __restrict__ nan_count) {
  __shared__ float red[16];
  const int D = t.D;
  float part = 0.f;
  for (int64_t r = threadIdx.x; r < b; r += 1024) {
    const int64_t c = target[r], h = hist[r * hist_ld];
    float acc = 0.f;
    for (int d = 0; d < D; ++d) acc = fmaf(t.qt[c * D + d], t.kh[h * D + d], acc);
    part += expf(acc / t.scale);
  }
  part = wave_sum(part);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  float S = 0.f;
  for (int w = 0; w < 16; ++w) S += red[w];
  const float Sb = (t.beta == 0.5f) ? sqrtf(S) : powf(S, t.beta);
  int nan = 0;
  for (int64_t r = threadIdx.x; r < b; r += 1024) {
    const int64_t c = target[r], h = hist[r * hist_ld];
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(t.vh[h * D + d], t.xt[c * D + d], s);
    const float logit = (h != c) ? s * (S / Sb) : __builtin_nanf("");   // 0/0 when masked
    out[r] = sigmoid ? sigm(logit) : logit;
    nan += (logit != logit);
  }
  if (nan_count && nan) atomicAdd(nan_count, nan);
}

// ------------------------------------------------------------------ pair tables
// E[j, c] = exp(qt_c . kh_{items[j]} / scale), ES[j, c] = E[j, c] * (vh_{items[j]} . xt_c) for
// the column block [col0, col0 + cols). 64 x 64 (j, c) tile per 256-thread workgroup, 4 x 4 per
// thread, D staged through LDS in 32-wide slices: two fp32 GEMMs with an exp epilogue.
constexpr int TJ = 64, TC = 64, TK = 32;
__global__ void __launch_bounds__(256)
dot_pair_table_kernel(Tabs t, const int64_t* __restrict__ items, int64_t J, int64_t col0,
                      int64_t cols, float* __restrict__ E, float* __restrict__ ES, int64_t ld) {
  __shared__ float sk[TK][TJ + 4], sv[TK][TJ + 4], sq[TK][TC + 4], sx[TK][TC + 4];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;   // c = tx*4.., j = ty*4..
  const int64_t jb = int64_t(blockIdx.y) * TJ, cb = int64_t(blockIdx.x) * TC;
  const int D = t.D;
  float a[4][4] = {}, s[4][4] = {};
  for (int k0 = 0; k0 < D; k0 += TK) {
    for (int f = threadIdx.x; f < TJ * TK; f += 256) {
      const int jj = f / TK, kk = f % TK;
      const int64_t j = jb + jj;
      float kv = 0.f, vv = 0.f;
      if (j < J && k0 + kk < D) {
        const int64_t it = items[j];
        kv = t.kh[it * D + k0 + kk];
        vv = t.vh[it * D + k0 + kk];
      }
      sk[kk][jj] = kv;
      sv[kk][jj] = vv;
    }
    for (int f = threadIdx.x; f < TC * TK; f += 256) {
      const int cc = f / TK, kk = f % TK;
      const int64_t c = cb + cc;
      float qv = 0.f, xv = 0.f;
      if (c < cols && k0 + kk < D) {
        qv = t.qt[(col0 + c) * D + k0 + kk];
        xv = t.xt[(col0 + c) * D + k0 + kk];
      }
      sq[kk][cc] = qv;
      sx[kk][cc] = xv;
    }
    __syncthreads();
    const int kn = std::min(TK, D - k0);
    for (int kk = 0; kk < kn; ++kk) {
      float kr[4], vr[4], qr[4], xr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        kr[i] = sk[kk][ty * 4 + i];
        vr[i] = sv[kk][ty * 4 + i];
        qr[i] = sq[kk][tx * 4 + i];
        xr[i] = sx[kk][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a[i][q] = fmaf(kr[i], qr[q], a[i][q]);
          s[i][q] = fmaf(vr[i], xr[q], s[i][q]);
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t j = jb + ty * 4 + i;
    if (j >= J) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t c = cb + tx * 4 + q;
      if (c >= cols) continue;
      const float e = expf(a[i][q] / t.scale);
      E[j * ld + c] = e;
      ES[j * ld + c] = e * s[i][q];
    }
  }
}

// ------------------------------------------------------------------ one-item-history users
// new4_validation's chunk k holds candidates i in [1024k, 1024k + 1024) of the complement list
// (ascending ids without the history item h: c = i + (i >= h)); every score in it is
// sigmoid(s_c * S_k / S_k^beta), S_k = sum over the chunk of e_c. One workgroup per (chunk, user).
__global__ void __launch_bounds__(1024)
dot_single_fixup_kernel(Tabs t, int64_t P, const int64_t* __restrict__ indptr,
                        const int64_t* __restrict__ indices, const int32_t* __restrict__ users,
                        int64_t col0, int64_t cols, float* __restrict__ scores, int64_t score_ld,
                        int64_t score_col0) {
  __shared__ float red[16];
  const int64_t slot = blockIdx.y;
  const int64_t u = users[slot];
  if (indptr[u + 1] - indptr[u] != 1) return;   // workgroup-uniform
  const int64_t h = indices[indptr[u]];
  const int64_t i = int64_t(blockIdx.x) * 1024 + threadIdx.x;
  const int64_t c = i + (i >= h);
  const bool live = i < P - 1;
  const int D = t.D;
  float e = 0.f;
  if (live) {
    float acc = 0.f;
    for (int d = 0; d < D; ++d) acc = fmaf(t.qt[c * D + d], t.kh[h * D + d], acc);
    e = expf(acc / t.scale);
  }
  float part = wave_sum(e);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  float S = 0.f;
  for (int w = 0; w < 16; ++w) S += red[w];
  if (!live || c < col0 || c >= col0 + cols) return;
  const float Sb = (t.beta == 0.5f) ? sqrtf(S) : powf(S, t.beta);
  float s = 0.f;
  for (int d = 0; d < D; ++d) s = fmaf(t.vh[h * D + d], t.xt[c * D + d], s);
  scores[slot * score_ld + (c - score_col0)] = sigm(s * (S / Sb));
}

int check_tabs(const nais_dot_tables_t* t) {
  if (!t) return nais_internal_fail(NAIS_E_INVALID, "NULL tables");
  if (t->embed_dim <= 0 || t->embed_dim > 128 || t->num_pois <= 0 || !(t->scale_dim > 0.f))
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "embed_dim must be 1..128, num_pois > 0, scale_dim > 0");
  if (!t->xh || !t->xt || !t->qt || !t->kh || !t->vh)
    return nais_internal_fail(NAIS_E_INVALID, "NULL table pointer");
  return NAIS_OK;
}

Tabs make_tabs(const nais_dot_tables_t* t) {
  Tabs r;
  r.D = t->embed_dim;
  r.beta = t->beta;
  r.scale = sqrtf(t->scale_dim);   // torch.sqrt(torch.tensor(self.embed_size)) in f32
  r.xh = t->xh; r.xt = t->xt; r.qt = t->qt; r.kh = t->kh; r.vh = t->vh;
  return r;
}

}  // namespace

extern "C" {

int32_t nais_linear_rows(const float* x, int64_t x_ld, int64_t rows, int32_t din, const float* w,
                         const float* b, int32_t dout, float* y, int64_t y_ld, void* stream) {
  if (rows < 0 || din <= 0 || dout <= 0 || dout > 256 || x_ld < din || y_ld < dout)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape (dout <= 256)");
  if (size_t(din) * dout * sizeof(float) > 160 * 1024)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "din * dout too large for LDS");
  if (rows == 0) return NAIS_OK;
  if (!x || !w || !y) return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  static bool once = (hipFuncSetAttribute(reinterpret_cast<const void*>(linear_rows_kernel),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
                      true);
  (void)once;
  const int rows_per = 256 / dout;
  const int64_t blocks = std::min<int64_t>((rows + rows_per - 1) / rows_per, 8192);
  hipLaunchKernelGGL(linear_rows_kernel, dim3((unsigned)blocks), dim3(256),
                     size_t(din) * dout * sizeof(float), reinterpret_cast<hipStream_t>(stream), x,
                     x_ld, rows, (int)din, w, b, (int)dout, y, y_ld);
  return nais_internal_check_launch("linear_rows_kernel");
}

int32_t nais_dot_forward(const nais_dot_tables_t* tables, const int64_t* hist, int64_t b, int64_t n,
                         int64_t hist_ld, const int64_t* target, float* out, int32_t* nan_count,
                         int32_t flags, void* stream) {
  int rc = check_tabs(tables);
  if (rc) return rc;
  if (b < 0 || n < 0 || (n > 0 && hist_ld < n)) return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (b == 0) return NAIS_OK;
  if (!target || !out || (n > 0 && !hist)) return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  const Tabs t = make_tabs(tables);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int sig = (flags & NAIS_FLAG_SIGMOID) ? 1 : 0;
  if (n == 1) {
    hipLaunchKernelGGL(dot_forward_single_kernel, dim3(1), dim3(1024), 0, st, t, hist, b, hist_ld,
                       target, out, sig, nan_count);
    return nais_internal_check_launch("dot_forward_single_kernel");
  }
  hipLaunchKernelGGL(dot_forward_kernel, dim3((unsigned)((b + FW - 1) / FW)), dim3(FW * 64), 0, st, t,
                     hist, b, n, hist_ld, target, out, sig, nan_count);
  return nais_internal_check_launch("dot_forward_kernel");
}

int32_t nais_dot_pair_table(const nais_dot_tables_t* tables, const int64_t* items, int64_t num_items,
                            int64_t col0, int64_t cols, float* e, float* es, int64_t ld,
                            void* stream) {
  int rc = check_tabs(tables);
  if (rc) return rc;
  if (num_items < 0 || cols < 0 || col0 < 0 || col0 + cols > tables->num_pois || ld < cols)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (num_items == 0 || cols == 0) return NAIS_OK;
  if (!items || !e || !es) return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  if ((num_items + TJ - 1) / TJ > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "too many items");
  hipLaunchKernelGGL(dot_pair_table_kernel, dim3((unsigned)((cols + TC - 1) / TC), (unsigned)((num_items + TJ - 1) / TJ)),
                     dim3(256), 0, reinterpret_cast<hipStream_t>(stream), make_tabs(tables), items,
                     num_items, col0, cols, e, es, ld);
  return nais_internal_check_launch("dot_pair_table_kernel");
}

int32_t nais_dot_single_fixup(const nais_dot_tables_t* tables, const int64_t* indptr,
                              const int64_t* indices, const int32_t* users, int64_t num_users,
                              int64_t col0, int64_t cols, float* scores, int64_t score_ld,
                              int64_t score_col0, void* stream) {
  int rc = check_tabs(tables);
  if (rc) return rc;
  const int64_t P = tables->num_pois;
  if (num_users < 0 || col0 < score_col0 || cols < 0 || col0 + cols > P ||
      score_ld < col0 + cols - score_col0)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (num_users == 0 || cols == 0 || P < 2) return NAIS_OK;
  if (!indptr || !indices || !users || !scores) return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  if (num_users > 65535) return nais_internal_fail(NAIS_E_UNSUPPORTED, "num_users > 65535 per call");
  const int64_t chunks = (P - 1 + 1023) / 1024;
  hipLaunchKernelGGL(dot_single_fixup_kernel, dim3((unsigned)chunks, (unsigned)num_users), dim3(1024), 0,
                     reinterpret_cast<hipStream_t>(stream), make_tabs(tables), P, indptr, indices,
                     users, col0, cols, scores, score_ld, score_col0);
  return nais_internal_check_launch("dot_single_fixup_kernel");
}

}  // extern "C"
