// nais_new4.hip -- per-POI context tables of the New4 family (model.py:1169-2228).
//
// Every table-based member of the family (New4, New4_padding, all_in_out, nearPOI_embedding,
// no_POI_emb, transform_ingoing_outgoing, only_area_not_inout) first pools each POI's near-POI
// list with a one-query attention (its self_attention, e.g. model.py:1272-1295):
//   x_k = KV[near[p][k]] (k < K),  q = Q[near[p][0]]                         (rows of width d)
//   key_k = Wk x_k + bk, val_k = Wv x_k + bv, q = Wq q + bq   (transform_* only; else identity)
//   r_p = softmax(q . reshape(key, [d, K]) / sqrt(scale_dim)) @ val
// (reshape, not transpose: the [K, d] keys are reinterpreted as [d, K], as the reference does),
// then runs NAIS_basic's attention over rows concatenated from embedding columns and these r.
// nais_near_attention computes r for every POI straight into a column range of the caller's
// [P, D] row table (one 64-lane workgroup per POI, the K x d slices in LDS); the scoring is then
// the basic variant over the two row tables. nais_new4_tables = New4's two pools + its layout.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "nais.h"
#include "nais_internal.h"

namespace {

struct Lin {
  const float* w;   // [d, d] row-major (nn.Linear.weight) or NULL (identity)
  const float* b;   // [d]
};

// y = W x + b (torch Linear) for one d-vector in LDS, lanes over outputs
__device__ __forceinline__ void linear_row(const Lin& l, const float* x, float* y, int d, int lane) {
  for (int o = lane; o < d; o += 64) {
    float acc = 0.f;
    for (int i = 0; i < d; ++i) acc = fmaf(x[i], l.w[o * d + i], acc);
    y[o] = acc + (l.b ? l.b[o] : 0.f);
  }
}

__global__ void __launch_bounds__(64)
near_attention_kernel(const float* __restrict__ qsrc, const float* __restrict__ kvsrc, int d,
                      const int64_t* __restrict__ near, int K, Lin lq, Lin lk, Lin lv,
                      float scale_dim, float* __restrict__ out, int64_t out_ld) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x;
  const int64_t p = blockIdx.x;
  float* xs = sm;                 // [K][d] raw rows
  float* ks = xs + K * d;         // [K][d] keys (== xs without a projection)
  float* vs = ks + K * d;         // [K][d] values
  float* qv = vs + K * d;         // [2][d] query (raw, projected)
  float* lg = qv + 2 * d;         // [K] logits -> weights
  for (int f = lane; f < K * d; f += 64) {
    const int k = f / d, c = f % d;
    xs[f] = kvsrc[near[p * K + k] * d + c];
  }
  for (int c = lane; c < d; c += 64) qv[c] = qsrc[near[p * K] * d + c];
  __syncthreads();
  const float* q = qv;
  const float* keys = xs;
  const float* vals = xs;
  if (lq.w) {
    linear_row(lq, qv, qv + d, d, lane);
    q = qv + d;
  }
  if (lk.w) {
    for (int k = 0; k < K; ++k) linear_row(lk, xs + k * d, ks + k * d, d, lane);
    keys = ks;
  }
  if (lv.w) {
    for (int k = 0; k < K; ++k) linear_row(lv, xs + k * d, vs + k * d, d, lane);
    vals = vs;
  }
  __syncthreads();
  const float scale = sqrtf(scale_dim);   // torch.sqrt(torch.tensor(embed_size / 4 or / 2)), f32
  for (int b = lane; b < K; b += 64) {
    float acc = 0.f;
    for (int a = 0; a < d; ++a) acc = fmaf(q[a], keys[a * K + b], acc);
    lg[b] = acc / scale;
  }
  __syncthreads();
  if (lane == 0) {                 // nn.Softmax(dim=-1) over the K near POIs
    float mx = -INFINITY;
    for (int b = 0; b < K; ++b) mx = fmaxf(mx, lg[b]);
    float s = 0.f;
    for (int b = 0; b < K; ++b) {
      lg[b] = expf(lg[b] - mx);
      s += lg[b];
    }
    for (int b = 0; b < K; ++b) lg[b] = lg[b] / s;
  }
  __syncthreads();
  for (int c = lane; c < d; c += 64) {
    float acc = 0.f;
    for (int b = 0; b < K; ++b) acc = fmaf(lg[b], vals[b * d + c], acc);
    out[p * out_ld + c] = acc;
  }
}

// dst[p, col0 + c] = src[p, c] for c < d (embedding columns / pools into the row tables)
__global__ void copy_cols_kernel(const float* __restrict__ src, int64_t src_ld, int d, int64_t P,
                                 float* __restrict__ dst, int64_t ld, int col0) {
  const int64_t f = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (f >= P * d) return;
  const int64_t p = f / d;
  const int c = int(f % d);
  dst[p * ld + col0 + c] = src[p * src_ld + c];
}

}  // namespace

extern "C" {

int32_t nais_near_attention(const float* query_src, const float* kv_src, int64_t num_pois,
                            int32_t dim, const int64_t* near_pois, int32_t num_near,
                            const float* wq, const float* bq, const float* wk, const float* bk,
                            const float* wv, const float* bv, float scale_dim, float* out,
                            int64_t out_ld, void* stream) {
  if (num_pois <= 0 || dim <= 0 || num_near <= 0 || out_ld < dim || !(scale_dim > 0.f))
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (!query_src || !kv_src || !near_pois || !out) return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  if (num_pois > 0x7fffffffll) return nais_internal_fail(NAIS_E_UNSUPPORTED, "num_pois too large");
  const size_t lds = (size_t(3) * num_near * dim + 2 * dim + num_near) * sizeof(float);
  if (lds > 160 * 1024) return nais_internal_fail(NAIS_E_UNSUPPORTED, "num_near * dim too large for LDS");
  static bool once = (hipFuncSetAttribute(reinterpret_cast<const void*>(near_attention_kernel),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
                      true);
  (void)once;
  hipLaunchKernelGGL(near_attention_kernel, dim3((unsigned)num_pois), dim3(64), lds,
                     reinterpret_cast<hipStream_t>(stream), query_src, kv_src, (int)dim, near_pois,
                     (int)num_near, Lin{wq, bq}, Lin{wk, bk}, Lin{wv, bv}, scale_dim, out, out_ld);
  return nais_internal_check_launch("near_attention_kernel");
}

int32_t nais_copy_columns(const float* src, int64_t src_ld, int64_t rows, int32_t dim, float* dst,
                          int64_t dst_ld, int32_t dst_col0, void* stream) {
  if (rows < 0 || dim <= 0 || src_ld < dim || dst_col0 < 0 || dst_ld < dst_col0 + dim)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (rows == 0) return NAIS_OK;
  if (!src || !dst) return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  const int64_t n = rows * dim;
  hipLaunchKernelGGL(copy_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), src, src_ld, (int)dim, rows, dst, dst_ld,
                     (int)dst_col0);
  return nais_internal_check_launch("copy_cols_kernel");
}

int32_t nais_new4_tables(const float* embed_history, const float* embed_target,
                         const float* embed_ingoing, const float* embed_outgoing,
                         int64_t num_pois, int32_t embed_size, const int64_t* near_pois,
                         int32_t num_near, float* ext_history, float* ext_target, void* stream) {
  if (num_pois <= 0 || embed_size <= 0 || embed_size % 4 != 0 || num_near <= 0)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape (embed_size must be a multiple of 4)");
  if (!embed_history || !embed_target || !embed_ingoing || !embed_outgoing || !near_pois ||
      !ext_history || !ext_target)
    return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  const int D = embed_size, half = D / 2, d4 = D / 4;
  const float sd = float(embed_size) / 4.f;
  int rc;
  // history rows [E_hist | in | out], target rows [E_tgt | out | in] (model.py:1215-1222)
  if ((rc = nais_copy_columns(embed_history, half, num_pois, half, ext_history, D, 0, stream))) return rc;
  if ((rc = nais_copy_columns(embed_target, half, num_pois, half, ext_target, D, 0, stream))) return rc;
  // result_out: q = in[0], keys/values = out ; result_in: q = out[0], keys/values = in
  if ((rc = nais_near_attention(embed_ingoing, embed_outgoing, num_pois, d4, near_pois, num_near,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, sd,
                                ext_history + half + d4, D, stream)))
    return rc;
  if ((rc = nais_near_attention(embed_outgoing, embed_ingoing, num_pois, d4, near_pois, num_near,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, sd,
                                ext_history + half, D, stream)))
    return rc;
  // the target rows hold the same two pools, swapped
  if ((rc = nais_copy_columns(ext_history + half + d4, D, num_pois, d4, ext_target, D, half, stream)))
    return rc;
  if ((rc = nais_copy_columns(ext_history + half, D, num_pois, d4, ext_target, D, half + d4, stream)))
    return rc;
  return NAIS_OK;
}

}  // extern "C"
