// Global-memory loads through pointers the compiler cannot place (device code only).
//
// A pointer loaded from a problem descriptor in memory is generic (flat) to the compiler.
// A flat load counts against the LDS counter as well as the vector-memory one, so a
// prefetch through one stalls the wave's next LDS wait until its data arrives from HBM,
// and an LDS-heavy loop around it loses the overlap it was written for.  Every buffer the
// kernels reach through such pointers is device or host-mapped global memory: ldg / gst
// access it through a global address-space pointer, so the compiler emits global loads
// and stores.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

namespace orbx {

template <typename T>
__device__ __forceinline__ T ldg(const T* p) {
    if constexpr (std::is_scalar<T>::value) {
        return *(const __attribute__((address_space(1))) T*)p;
    } else {
        // structs: word loads (the compiler merges them), reassembled in registers
        static_assert(sizeof(T) % 4 == 0, "whole words");
        constexpr int kW = (int)(sizeof(T) / 4);
        const __attribute__((address_space(1))) int* g = (const __attribute__((address_space(1))) int*)p;
        int w[kW];
#pragma unroll
        for (int i = 0; i < kW; i++) w[i] = g[i];
        T r;
        __builtin_memcpy(&r, w, sizeof(T));
        return r;
    }
}

template <typename T>
__device__ __forceinline__ void gst(T* p, T v) {
    static_assert(std::is_scalar<T>::value, "scalar stores");
    *(__attribute__((address_space(1))) T*)p = v;
}

}  // namespace orbx
