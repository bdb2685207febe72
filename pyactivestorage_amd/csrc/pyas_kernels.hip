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

// Batched un-shuffle of whole chunks (pyas_unshuffle_chunks): block (c, j)
// of chunk c takes groups of 4 elements; a lane reads one dword from each of
// the ES byte planes (a wave reads 256 contiguous bytes of every plane) and
// writes its 4 elements as ES dwords.  Chunks whose planes are not dword
// aligned, and the n % 4 tail, go byte by byte.
template <int ES>
__global__ __launch_bounds__(kBlock) void k_unshuffle_chunks(const uint8_t *src, const int64_t *soff,
                                                             uint8_t *dst, const int64_t *doff,
                                                             int64_t nbytes, int64_t bpc) {
    const int64_t c = blockIdx.x / bpc, j = blockIdx.x - c * bpc;
    const uint8_t *s = src + soff[c];
    uint8_t *d = dst + doff[c];
    const int64_t n = nbytes / ES;
    const bool vec = (((uintptr_t)s | (uintptr_t)d) & 3) == 0 && (n & 3) == 0;
    const int64_t groups = vec ? n / 4 : 0;
    for (int64_t g = j * kBlock + threadIdx.x; g < groups; g += bpc * kBlock) {
        uint32_t w[ES];
#pragma unroll
        for (int b = 0; b < ES; ++b) w[b] = *reinterpret_cast<const uint32_t *>(s + b * n + g * 4);
        uint32_t o[ES];
#pragma unroll
        for (int q = 0; q < ES; ++q) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {        // output byte 4q + t = element k, plane b
                const int ob = 4 * q + t, k = ob / ES, b = ob - k * ES;
                v |= ((w[b] >> (8 * k)) & 0xffu) << (8 * t);
            }
            o[q] = v;
        }
        uint32_t *dp = reinterpret_cast<uint32_t *>(d + g * 4 * ES);
#pragma unroll
        for (int q = 0; q < ES; ++q) dp[q] = o[q];
    }
    for (int64_t q = groups * 4 * ES + j * kBlock + threadIdx.x; q < nbytes; q += bpc * kBlock) {
        if (q < n * ES) {
            const int64_t i = q / ES, b = q - i * ES;
            d[q] = s[b * n + i];
        } else {
            d[q] = s[q];
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

hipError_t launch_combine_grid(int dtype, const pyas_partial *in, const pyas_grid &g, const CombineTie &ct,
                               int64_t n_out, int64_t n_layers, uint32_t flags,
                               pyas_partial *out, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_combine_grid_t<T>(in, g, ct, n_out, n_layers, flags, out, st));
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

hipError_t launch_tie_chunks(int dtype, const TieChunkArgs &a, int64_t grid, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_tie_chunks_t<T>(a, grid, st));
    return hipErrorInvalidValue;
}

hipError_t launch_tie_gate(int dtype, const pyas_partial *fin, int64_t n, uint32_t which, uint32_t *gate,
                           hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_tie_gate_t<T>(fin, n, which, gate, st));
    return hipErrorInvalidValue;
}

hipError_t launch_tie_grid(int dtype, const TieGridArgs &a, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_tie_grid_t<T>(a, st));
    return hipErrorInvalidValue;
}

hipError_t launch_tie_pick(int dtype, const pyas_partial *parts, int64_t n, uint32_t which, int64_t base,
                           const TieCall &call, const TieRule &t, uint64_t *keys, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_tie_pick_t<T>(parts, n, which, base, call, t, keys, st));
    return hipErrorInvalidValue;
}

hipError_t launch_tie_finalize(int dtype, const uint64_t *keys, int64_t n_out, int32_t n_sets, const TieCall &call,
                               const TieRule &t, uint32_t which, pyas_partial *fin, hipStream_t st) {
    PYAS_DISPATCH_T(dtype, return launch_tie_finalize_t<T>(keys, n_out, n_sets, call, t, which, fin, st));
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

hipError_t launch_unshuffle_chunks(const void *src, const int64_t *soff, void *dst, const int64_t *doff,
                                   int64_t n_chunks, int64_t nbytes, int64_t es, hipStream_t st) {
    int64_t bpc = (nbytes / 16 + kBlock - 1) / kBlock;   // ~16 output bytes per lane
    if (bpc > 64) bpc = 64;
    if (bpc < 1) bpc = 1;
    const dim3 g((unsigned)(n_chunks * bpc)), b(kBlock);
    const uint8_t *s = (const uint8_t *)src;
    uint8_t *d = (uint8_t *)dst;
    if (es == 2) hipLaunchKernelGGL(k_unshuffle_chunks<2>, g, b, 0, st, s, soff, d, doff, nbytes, bpc);
    else if (es == 4) hipLaunchKernelGGL(k_unshuffle_chunks<4>, g, b, 0, st, s, soff, d, doff, nbytes, bpc);
    else if (es == 8) hipLaunchKernelGGL(k_unshuffle_chunks<8>, g, b, 0, st, s, soff, d, doff, nbytes, bpc);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace pyas
