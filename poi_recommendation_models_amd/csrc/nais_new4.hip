// nais_new4.hip -- per-POI context tables of the New4 family (model.py:1169-1306).
//
// New4.forward (model.py:1212-1222) first turns every POI's near-POI list into two context
// vectors with a one-query attention (self_attention, model.py:1272-1295):
//   in  = Ein[near[p]]  [K, d4],  out = Eout[near[p]] [K, d4]          (d4 = embed_size / 4)
//   result_out = softmax(in[0] . reshape(out, [d4, K]) / sqrt(d4)) @ out
//   result_in  = softmax(out[0] . reshape(in,  [d4, K]) / sqrt(d4)) @ in
// (reshape, not transpose: the [K, d4] rows are reinterpreted as [d4, K], as the reference does),
// then runs NAIS_basic's attention_network on the concatenations
//   history row = [E_hist[j] | result_in[j] | result_out[j]],  target row = [E_tgt[c] | result_out[c] | result_in[c]].
// So the scoring itself is the basic variant over two [P, D] tables; this kernel builds them
// (one 64-lane workgroup per POI, the K x d4 slices staged in LDS), and the catalog / forward
// kernels consume them unchanged.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "nais.h"
#include "nais_internal.h"

namespace {

__global__ void __launch_bounds__(64)
new4_tables_kernel(const float* __restrict__ eh, const float* __restrict__ et,
                   const float* __restrict__ ein, const float* __restrict__ eout, int64_t P, int D,
                   const int64_t* __restrict__ near, int K, float* __restrict__ xh,
                   float* __restrict__ xt) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x;
  const int64_t p = blockIdx.x;
  const int d4 = D / 4, half = D / 2;
  float* sin_ = sm;                 // [K][d4] ingoing rows
  float* sout = sin_ + K * d4;      // [K][d4] outgoing rows
  float* lg = sout + K * d4;        // [2][K] logits -> softmax weights (0: out, 1: in)
  for (int f = lane; f < K * d4; f += 64) {
    const int k = f / d4, c = f % d4;
    const int64_t id = near[p * K + k];
    sin_[f] = ein[id * d4 + c];
    sout[f] = eout[id * d4 + c];
  }
  __syncthreads();
  const float scale = sqrtf(float(d4));   // torch.sqrt(torch.tensor(embed_size / 4)), float32
  for (int b = lane; b < 2 * K; b += 64) {
    const bool in = b >= K;
    const int bb = in ? b - K : b;
    const float* q = in ? sout : sin_;    // query: row 0 of the other table
    const float* kf = in ? sin_ : sout;   // [K][d4] read as [d4][K]
    float acc = 0.f;
    for (int a = 0; a < d4; ++a) acc = fmaf(q[a], kf[a * K + bb], acc);
    lg[b] = acc / scale;
  }
  __syncthreads();
  if (lane < 2) {                          // softmax over K (nn.Softmax(dim=-1))
    float* l = lg + lane * K;
    float mx = -INFINITY;
    for (int b = 0; b < K; ++b) mx = fmaxf(mx, l[b]);
    float s = 0.f;
    for (int b = 0; b < K; ++b) {
      l[b] = expf(l[b] - mx);
      s += l[b];
    }
    for (int b = 0; b < K; ++b) l[b] = l[b] / s;
  }
  __syncthreads();
  for (int f = lane; f < half; f += 64) {
    xh[p * D + f] = eh[p * half + f];
    xt[p * D + f] = et[p * half + f];
  }
  for (int c = lane; c < 2 * d4; c += 64) {
    const bool in = c >= d4;
    const int cc = in ? c - d4 : c;
    const float* w = lg + (in ? K : 0);
    const float* v = in ? sin_ : sout;
    float acc = 0.f;
    for (int b = 0; b < K; ++b) acc = fmaf(w[b], v[b * d4 + cc], acc);
    // history row: [.. | in | out], target row: [.. | out | in]
    xh[p * D + half + (in ? 0 : d4) + cc] = acc;
    xt[p * D + half + (in ? d4 : 0) + cc] = acc;
  }
}

}  // namespace

extern "C" int32_t nais_new4_tables(const float* embed_history, const float* embed_target,
                                    const float* embed_ingoing, const float* embed_outgoing,
                                    int64_t num_pois, int32_t embed_size, const int64_t* near_pois,
                                    int32_t num_near, float* ext_history, float* ext_target,
                                    void* stream) {
  if (num_pois <= 0 || embed_size <= 0 || embed_size % 4 != 0 || num_near <= 0)
    return nais_internal_fail(NAIS_E_INVALID, "bad shape (embed_size must be a multiple of 4)");
  if (!embed_history || !embed_target || !embed_ingoing || !embed_outgoing || !near_pois ||
      !ext_history || !ext_target)
    return nais_internal_fail(NAIS_E_INVALID, "NULL pointer");
  if (num_pois > 0x7fffffffll) return nais_internal_fail(NAIS_E_UNSUPPORTED, "num_pois too large");
  const size_t lds = (size_t(2) * num_near * (embed_size / 4) + size_t(2) * num_near) * sizeof(float);
  if (lds > 160 * 1024) return nais_internal_fail(NAIS_E_UNSUPPORTED, "num_near * embed_size too large for LDS");
  static bool once = (hipFuncSetAttribute(reinterpret_cast<const void*>(new4_tables_kernel),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
                      true);
  (void)once;
  hipLaunchKernelGGL(new4_tables_kernel, dim3((unsigned)num_pois), dim3(64), lds,
                     reinterpret_cast<hipStream_t>(stream), embed_history, embed_target,
                     embed_ingoing, embed_outgoing, num_pois, (int)embed_size, near_pois,
                     (int)num_near, ext_history, ext_target);
  return nais_internal_check_launch("new4_tables_kernel");
}
