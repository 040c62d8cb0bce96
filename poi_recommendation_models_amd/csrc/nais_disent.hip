// nais_disent.hip -- NAIS_region_distance_disentangled_Embedding (model.py:409-541).
//
// Two NAIS attentions side by side, one over the POI embeddings and one over the region
// embeddings (both embed_size wide), sharing an additive distance term (model.py:490-518):
//   l_j  = attn_layer2(relu(attn_layer1(h_j (.) t)))            r_j = region_attn_layer2(relu(
//                                                                      region_attn_layer1(g_j (.) g_t)))
//   d_j  = sum_e embed_distance[0][e] * target_distance[j]       (index 0 for every entry, :488-491)
//   a_j  = m_j exp(l_j + d_j) / (sum m exp(l + d))^beta          rho_j likewise with r_j
//   logit = sum_j a_j (h_j . t) + rho_j (g_j . g_t)               (cat + bmm, model.py:522-527)
// No dropout in this model. forward_kernel: one 64-lane workgroup per row; for every history
// entry the two D-wide products are staged in LDS and each lane evaluates up to two hidden units
// of each MLP (H <= 128), wave-reduced.
//
// nais_pair_distances: run.py:326-333's target_dist for a batch -- powerLaw.dist (haversine km,
// float64, reference operation order; nais_geo.h) between every target and history POI, rounded
// to float32 as torch.tensor(..., dtype=torch.float32) does.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "nais.h"
#include "nais_geo.h"
#include "nais_internal.h"

namespace {

__device__ __forceinline__ float wsum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

struct DP {
  int D, H;
  float beta;
  const float *eh, *et, *er, *ed, *w1, *b1, *w2, *rw1, *rb1, *rw2;
};

// w2 . relu(W1 x + b1) for the lanes' hidden units (x in LDS), wave-reduced
__device__ __forceinline__ float mlp(const float* x, const float* w1, const float* b1,
                                     const float* w2, int D, int H, int lane) {
  float part = 0.f;
  for (int i = lane; i < H; i += 64) {
    float a = 0.f;
    const float* wr = w1 + int64_t(i) * D;
    for (int d = 0; d < D; ++d) a = fmaf(wr[d], x[d], a);
    a += b1[i];
    part = fmaf(w2[i], nais_relu(a), part);
  }
  return wsum(part);
}

__global__ void __launch_bounds__(64)
disent_forward_kernel(DP p, const int64_t* __restrict__ hist, int64_t n, int64_t hist_ld,
                      const int64_t* __restrict__ target, const int64_t* __restrict__ hreg,
                      int64_t hreg_ld, const int64_t* __restrict__ treg,
                      const float* __restrict__ tdist, int64_t dist_ld, float* __restrict__ out,
                      int sigmoid, int32_t* __restrict__ nan_count) {
  __shared__ float xs[128], xr[128];
  const int lane = threadIdx.x;
  const int64_t r = blockIdx.x;
  const int D = p.D, H = p.H;
  const int64_t c = target[r], gc = treg[r];
  float S1 = 0.f, N1 = 0.f, S2 = 0.f, N2 = 0.f;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t h = hist[r * hist_ld + j], g = hreg[r * hreg_ld + j];
    const float x = tdist[r * dist_ld + j];
    float dot1 = 0.f, dot2 = 0.f, dpart = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float hv = p.eh[h * D + d], tv = p.et[c * D + d];
      const float gv = p.er[g * D + d], gt = p.er[gc * D + d];
      xs[d] = hv * tv;
      xr[d] = gv * gt;
      dot1 = fmaf(hv, tv, dot1);
      dot2 = fmaf(gv, gt, dot2);
      dpart = fmaf(p.ed[d], x, dpart);
    }
    __syncthreads();
    const float l = mlp(xs, p.w1, p.b1, p.w2, D, H, lane);
    const float rr = mlp(xr, p.rw1, p.rb1, p.rw2, D, H, lane);
    const float dj = wsum(dpart);
    const float ht = wsum(dot1), gg = wsum(dot2);
    __syncthreads();
    const float m = (h != c) ? 1.f : 0.f;           // exp * mask: inf * 0 -> NaN as in torch
    const float e1 = expf(l + dj) * m, e2 = expf(rr + dj) * m;
    S1 += e1;
    N1 = fmaf(e1, ht, N1);
    S2 += e2;
    N2 = fmaf(e2, gg, N2);
  }
  float logit = 0.f;
  if (n > 0) {
    const float d1 = (p.beta == 0.5f) ? sqrtf(S1) : powf(S1, p.beta);
    const float d2 = (p.beta == 0.5f) ? sqrtf(S2) : powf(S2, p.beta);
    logit = N1 / d1 + N2 / d2;
  }
  if (lane == 0) {
    out[r] = sigmoid ? 1.0f / (1.0f + expf(-logit)) : logit;
    if (nan_count && logit != logit) atomicAdd(nan_count, 1);
  }
}

__global__ void pair_distances_kernel(const double* __restrict__ coords, const int64_t* __restrict__ hist,
                                      int64_t n, const int64_t* __restrict__ target, int64_t b,
                                      float* __restrict__ out) {
  const int64_t f = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (f >= b * n) return;
  const int64_t r = f / n, j = f % n;
  const int64_t c = target[r], h = hist[j];
  const Geo pc = make_geo(coords[2 * c], coords[2 * c + 1]);
  const Geo ph = make_geo(coords[2 * h], coords[2 * h + 1]);
  out[f] = float(ref_dist(pc, ph));   // dist(target, history), run.py:329-331
}

}  // namespace

extern "C" {

int32_t nais_disent_forward(const nais_disent_params_t* params, const int64_t* hist, int64_t b,
                            int64_t n, int64_t hist_ld, const int64_t* target,
                            const int64_t* hist_region, int64_t hist_region_ld,
                            const int64_t* target_region, const float* target_distance,
                            int64_t dist_ld, float* out, int32_t* nan_count, int32_t flags,
                            void* stream) {
  if (!params) return nais_internal_fail(NAIS_E_INVALID, "NULL params");
  const nais_disent_params_t& q = *params;
  if (q.embed_dim <= 0 || q.embed_dim > 128 || q.hidden <= 0 || q.hidden > 128)
    return nais_internal_fail(NAIS_E_UNSUPPORTED, "embed_dim and hidden must be 1..128");
  if (!q.embed_history || !q.embed_target || !q.embed_region || !q.embed_distance || !q.w1 ||
      !q.b1 || !q.w2 || !q.region_w1 || !q.region_b1 || !q.region_w2)
    return nais_internal_fail(NAIS_E_INVALID, "NULL parameter pointer");
  if (b < 0 || n < 0 || (n > 0 && (hist_ld < n || hist_region_ld < n || dist_ld < n)))
    return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (b == 0) return NAIS_OK;
  if (!target || !target_region || !out || (n > 0 && (!hist || !hist_region || !target_distance)))
    return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  if (b > 0x7fffffffll) return nais_internal_fail(NAIS_E_UNSUPPORTED, "b too large");
  DP p{q.embed_dim, q.hidden, q.beta, q.embed_history, q.embed_target, q.embed_region,
       q.embed_distance, q.w1, q.b1, q.w2, q.region_w1, q.region_b1, q.region_w2};
  hipLaunchKernelGGL(disent_forward_kernel, dim3((unsigned)b), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), p, hist, n, hist_ld, target, hist_region,
                     hist_region_ld, target_region, target_distance, dist_ld, out,
                     (flags & NAIS_FLAG_SIGMOID) ? 1 : 0, nan_count);
  return nais_internal_check_launch("disent_forward_kernel");
}

int32_t nais_pair_distances(const double* coords, const int64_t* hist, int64_t n,
                            const int64_t* target, int64_t b, float* out, void* stream) {
  if (b < 0 || n < 0) return nais_internal_fail(NAIS_E_INVALID, "bad shape");
  if (b == 0 || n == 0) return NAIS_OK;
  if (!coords || !hist || !target || !out) return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  const int64_t tot = b * n;
  hipLaunchKernelGGL(pair_distances_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), coords, hist, n, target, b, out);
  return nais_internal_check_launch("pair_distances_kernel");
}

}  // extern "C"
