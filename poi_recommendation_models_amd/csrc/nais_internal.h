// nais_internal.h -- declarations shared by the translation units of libnais_hip.so (not ABI).
#pragma once

#include <hip/hip_runtime.h>

// Records `msg` as the thread's nais_last_error() text and returns `code`.
__attribute__((visibility("hidden"))) int nais_internal_fail(int code, const char* msg);
// NAIS_E_HIP (with the HIP error text) if the last launch failed, else NAIS_OK.
__attribute__((visibility("hidden"))) int nais_internal_check_launch(const char* what);

// CUs a launch on `stream` may use: the popcount of its CU mask (hipExtStreamGetCUMask), the
// device's CU count for an unmasked stream; <= 0 on error. Sizes the work-queue grids, so a queue
// launch never leaves workgroups waiting for CUs held by another stream's launch.
__attribute__((visibility("hidden"))) int nais_internal_stream_cus(hipStream_t stream);

// ReLU that keeps NaN, as torch.relu (model.py:71): fmaxf / v_max_f32 would return 0 for a NaN.
__device__ __forceinline__ float nais_relu(float v) { return (v < 0.f) ? 0.f : v; }
