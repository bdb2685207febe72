// pyas_kernels.hip — dtype dispatch of the kernel launchers, and the
// standalone un-shuffle kernel.  The kernel templates are in pyas_kernels.hpp
// and are instantiated per dtype by pyas_inst.hip.
#include <hip/hip_runtime.h>

#include "pyas_device.hpp"
#include "pyas_internal.hpp"

namespace pyas {

__global__ __launch_bounds__(kBlock) void k_unshuffle(const uint8_t *src, uint8_t *dst, int64_t nbytes,
                                                      int64_t es) {
    const int64_t n = nbytes / es;
    const int64_t body = n * es;
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nbytes;
         q += (int64_t)gridDim.x * kBlock) {
        if (q < body) {
            const int64_t i = q / es, b = q - i * es;
            dst[q] = src[b * n + i];
        } else {
            dst[q] = src[q];
        }
    }
}

#define PYAS_DISPATCH_T(DT, CALL)                                  \
    switch (DT) {                                                  \
        case PYAS_I8: { using T = int8_t; CALL; } break;           \
        case PYAS_U8: { using T = uint8_t; CALL; } break;          \
        case PYAS_I16: { using T = int16_t; CALL; } break;         \
        case PYAS_U16: { using T = uint16_t; CALL; } break;        \
        case PYAS_I32: { using T = int32_t; CALL; } break;         \
        case PYAS_U32: { using T = uint32_t; CALL; } break;        \
        case PYAS_I64: { using T = int64_t; CALL; } break;         \
        case PYAS_U64: { using T = uint64_t; CALL; } break;        \
        case PYAS_F32: { using T = float; CALL; } break;           \
        case PYAS_F64: { using T = double; CALL; } break;          \
        default: return hipErrorInvalidValue;                      \
    }

hipError_t launch_reduce(int dtype, const ReduceArgs &a, bool shuf, bool bsw, bool masked,
                         int64_t grid, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_reduce_t<T>(a, shuf, bsw, masked, grid, st));
    return hipErrorInvalidValue;
}

hipError_t launch_finish(int dtype, const FinishArgs &f, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_finish_t<T>(f, st));
    return hipErrorInvalidValue;
}

hipError_t launch_combine(int dtype, const pyas_partial *in, int64_t n, int64_t seg, int64_t nblocks,
                          uint32_t flags, pyas_partial *out, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_combine_t<T>(in, n, seg, nblocks, flags, out, st));
    return hipErrorInvalidValue;
}

hipError_t launch_combine_segments(int dtype, const pyas_partial *in, const int64_t *index,
                                   const int64_t *seg, int64_t n_seg, uint32_t flags,
                                   pyas_partial *out, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_combine_segments_t<T>(in, index, seg, n_seg, flags, out, st));
    return hipErrorInvalidValue;
}

hipError_t launch_reduce_axes(int dtype, const AxesArgs &a, int64_t grid, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_axes_t<T>(a, grid, st));
    return hipErrorInvalidValue;
}

hipError_t launch_combine_grid(int dtype, const pyas_partial *in, const pyas_grid &g,
                               int64_t n_out, int64_t n_layers, uint32_t flags,
                               pyas_partial *out, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_combine_grid_t<T>(in, g, n_out, n_layers, flags, out, st));
    return hipErrorInvalidValue;
}

hipError_t launch_axes_dense(int dtype, const AxesArgs &a, bool masked, int64_t grid, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_axes_dense_t<T>(a, masked, grid, st));
    return hipErrorInvalidValue;
}

hipError_t launch_axes_fold(int dtype, const AxesArgs &a, const FoldGrid &g, bool masked, int64_t grid,
                            hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_axes_fold_t<T>(a, g, masked, grid, st));
    return hipErrorInvalidValue;
}

hipError_t launch_select(int dtype, const SelectArgs &a, int64_t grid, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_select_t<T>(a, grid, st));
    return hipErrorInvalidValue;
}

hipError_t launch_format(int dtype, const pyas_partial *in, int64_t n, int32_t method, void *values,
                         uint8_t *mask, int64_t *counts, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_format_t<T>(in, n, method, values, mask, counts, st));
    return hipErrorInvalidValue;
}

hipError_t launch_unshuffle(const void *src, void *dst, int64_t nbytes, int64_t es, hipStream_t st) {
    int64_t blocks = (nbytes + kBlock - 1) / kBlock;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_unshuffle, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                       (const uint8_t *)src, (uint8_t *)dst, nbytes, es);
    return hipGetLastError();
}

}  // namespace pyas
