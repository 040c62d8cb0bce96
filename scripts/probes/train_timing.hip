// train_timing.hip -- the TIMING build of nais_train.hip (never the product library): the per-phase
// cycle hooks of the training backward kernels (TSTART / TMARK / TFLUSH, no-ops in the product
// source) as s_memtime deltas summed per phase into g_train_cycles, and nais_debug_train_cycles()
// to read them. Results are unchanged; only the timing build carries the stamps.
//   python scripts/build_ab.py timing=nais_train.hip@scripts/probes/train_timing.hip
//   NAIS_HIP_LIB=build_ab/timing.so python scripts/train_phases.py --fused --D 128 --H 128
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ unsigned long long g_train_cycles[16];
#define TSTART() unsigned long long t_prev = __builtin_amdgcn_s_memtime(), t_acc[16] = {0}
#define TMARK(k)                                                   \
  do {                                                             \
    const unsigned long long t_now = __builtin_amdgcn_s_memtime(); \
    t_acc[k] += t_now - t_prev;                                    \
    t_prev = t_now;                                                \
  } while (0)
#define TFLUSH()                                                             \
  do {                                                                       \
    if ((threadIdx.x & 63) == 0)                                             \
      for (int q = 0; q < 16; ++q) atomicAdd(&g_train_cycles[q], t_acc[q]);  \
  } while (0)

#include "../../poi_recommendation_models_amd/csrc/nais_train.hip"

extern "C" int32_t nais_debug_train_cycles(unsigned long long* out16, int32_t reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_train_cycles), 16 * sizeof(unsigned long long)) !=
      hipSuccess)
    return NAIS_E_HIP;
  if (reset) {
    static const unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_train_cycles), z, sizeof(z)) != hipSuccess) return NAIS_E_HIP;
  }
  return NAIS_OK;
}
