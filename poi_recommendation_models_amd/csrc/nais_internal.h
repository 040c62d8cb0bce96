// nais_internal.h -- declarations shared by the translation units of libnais_hip.so (not ABI).
#pragma once

#include <hip/hip_runtime.h>

#include "nais.h"

// Records `msg` as the thread's nais_last_error() text and returns `code`.
__attribute__((visibility("hidden"))) int nais_internal_fail(int code, const char* msg);
// NAIS_E_HIP (with the HIP error text) if the last launch failed, else NAIS_OK.
__attribute__((visibility("hidden"))) int nais_internal_check_launch(const char* what);

// CUs a launch on `stream` may use: the popcount of its CU mask (hipExtStreamGetCUMask), the
// device's CU count for an unmasked stream; <= 0 on error. Sizes the work-queue grids, so a queue
// launch never leaves workgroups waiting for CUs held by another stream's launch.
__attribute__((visibility("hidden"))) int nais_internal_stream_cus(hipStream_t stream);

// The generic-shape scoring kernels (nais_generic.hip): any embed_dim <= 256, any hidden.
//   nais_gx_catalog: e == nullptr -- per-user catalog rows of users[0..nb) into scores (history
//   POIs -1, NaNs counted); else pair tables e / es [row][ld] of items[0..nitems) x columns
//   [col0, col0 + cols). nais_gx_forward: nais_forward's rows.
__attribute__((visibility("hidden"))) int nais_gx_catalog(
    const nais_params_t* params, const int64_t* indptr, const int64_t* indices, const int32_t* users,
    int nb, const int64_t* items, int64_t nitems, int64_t col0, int64_t cols, const int64_t* region_of,
    const double* coords, const double* latlon_mat, float* scores, int64_t score_ld,
    int32_t* nan_count, float* e, float* es, int64_t ld, hipStream_t st, int split = 0);
__attribute__((visibility("hidden"))) int nais_gx_forward(
    const nais_params_t* params, const int64_t* hist, int64_t b, int64_t n, int64_t hist_ld,
    const int64_t* target, const int64_t* hreg, int64_t hreg_ld, const int64_t* treg,
    const float* latlon, int64_t ll_ld, float* out, int32_t* nan_count, int32_t flags, hipStream_t st);

// Table words (v_perm_b32 selectors over {S0 = bits of e*s, S1 = bits of e}). The float tables
// store e and e*s as they are (NAIS_SEL_E); the split16 form (nais_pair_table_split) stores
//   hi = [top 16 bits of e*s | top 16 bits of e]  (NAIS_SEL_HI)  and  ex = (e, e*s) side by side,
// so hi alone gives both values truncated to 8 significant bits (relative error < 2^-7, toward
// zero; the bounded gather's phase 1) and one 8-byte ex read the exact pair (its refine).
constexpr uint32_t NAIS_SEL_E = 0x03020100u, NAIS_SEL_HI = 0x07060302u;

// ReLU that keeps NaN, as torch.relu (model.py:71): fmaxf / v_max_f32 would return 0 for a NaN.
__device__ __forceinline__ float nais_relu(float v) { return (v < 0.f) ? 0.f : v; }
