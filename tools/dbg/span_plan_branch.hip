// Round 6: the branch form of span_plan, reconstructed from
// the round-5 description (the pre-fix text was never committed): three
// branches, each storing all of the plan's per-form fields.  The kernel
// evaluates it beside the committed select form (pyas_kernels.hpp span_plan)
// for span_plan_dbg.hip's three selections; tools/dbg/Makefile builds it at
// -O0, -O1 and -O3 (and span_plan_host.cpp is the same text on the host
// under UBSan).
#include "../../pyactivestorage_amd/csrc/pyas_kernels.hpp"
#include <cstdio>
#include <cstring>
using namespace pyas;

template <typename T, bool SHUF>
__device__ __forceinline__ bool span_plan_branch(const ReduceArgs &a, const uint8_t *base, const Sel &s,
                                                 SpanPlan &sp) {
    constexpr int ES = sizeof(T);
    constexpr bool SH = SHUF && ES > 1;
    constexpr int NU = SH ? 16 : 16 / ES;
    if (a.tab.on[0] || a.tab.on[1] || a.chunk_elems >= (int64_t(1) << 31)) return false;
    if (SH && ((((uintptr_t)base) | (uint64_t)a.chunk_elems) & 15) != 0) return false;
    int k = -1;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d)
        if (d < a.ndim && k < 0 && !(s.step[d] == 1 && s.start[d] == 0 && (int64_t)s.cnt[d] == a.shape[d])) k = d;
    if (k < 0) return false;
    int64_t cs_k = 1, sk = 1, st_k = 0, cn_k = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d)
        if (d == k) { cs_k = a.cstride[d]; sk = s.step[d]; st_k = s.start[d]; cn_k = s.cnt[d]; }
    if (sk < 0) { st_k += (cn_k - 1) * sk; sk = -sk; }
    if (sk == 1 && (cn_k * cs_k + NU - 1) / NU + 1 <= kBlock) {   // a run of whole inner rows
        sp.kk = k;
        sp.m_in = (int32_t)(st_k * cs_k);
        sp.ext = (int32_t)(cn_k * cs_k);
        sp.istep = 1;
        sp.per_span = cn_k * cs_k;
    } else if (sk > 1 && k == a.ndim - 1) {                          // a strided innermost dim
        sp.kk = k;
        sp.m_in = (int32_t)st_k;
        sp.ext = (int32_t)((cn_k - 1) * sk + 1);
        sp.istep = (int32_t)sk;
        sp.per_span = cn_k;
    } else {                                                         // dim k enumerated too
        sp.kk = k + 1;
        sp.m_in = 0;
        sp.ext = (int32_t)cs_k;
        sp.istep = 1;
        sp.per_span = cs_k;
    }
    int64_t m0 = sp.m_in, nsp = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        if (d < sp.kk) {
            nsp *= s.cnt[d];
            if (s.cnt[d] > 0) m0 += sel_index(s, a.pool, d, 0) * a.cstride[d];
            if (s.cnt[d] > 1) {
                if (s.step[d] == 0 && d < sp.kk - 1) return false;
                const int64_t delta = (s.step[d] != 0 ? (int64_t)s.step[d] : 1) * a.cstride[d];
                if (SH ? (delta & 15) != 0 : ((delta * ES) & 15) != 0) return false;
            }
        }
    }
    sp.nspans = nsp;
    sp.off = SH ? (int32_t)(m0 & 15) : (int32_t)((((uintptr_t)base + (uint64_t)(m0 * ES)) & 15) / ES);
    const int64_t G = (sp.off + (int64_t)sp.ext + NU - 1) / NU;
    if (G < 1 || G > kBlock) return false;
    sp.G = (int32_t)G;
    sp.P = (int32_t)(kBlock / G);
    return true;
}

__global__ void k_dbg(ReduceArgs a, int32_t *out) {
    Sel s;
    load_sel(s, a.sel, blockIdx.x, a.ndim, a.shape);
    SpanPlan sp, sb;
    memset(&sp, 0, sizeof(sp));
    memset(&sb, 0, sizeof(sb));
    const bool ok = span_plan<float, false>(a, a.data, s, sp);
    const bool okb = span_plan_branch<float, false>(a, a.data, s, sb);
    if (threadIdx.x == 0) {
        int32_t *o = out + blockIdx.x * 16;
        o[0] = ok; o[1] = sp.kk; o[2] = sp.m_in; o[3] = sp.ext; o[4] = sp.istep; o[5] = sp.off; o[6] = (int32_t)sp.per_span;
        o[8] = okb; o[9] = sb.kk; o[10] = sb.m_in; o[11] = sb.ext; o[12] = sb.istep; o[13] = sb.off; o[14] = (int32_t)sb.per_span;
    }
}

int main() {
    const int n = 3;
    int32_t sel[n][PYAS_MAX_DIMS][3];
    int64_t shape[3] = {16, 16, 64};
    for (int c = 0; c < n; ++c)
        for (int d = 0; d < PYAS_MAX_DIMS; ++d) { sel[c][d][0] = 0; sel[c][d][1] = 1; sel[c][d][2] = d < 3 ? (int)shape[d] : 1; }
    // c0: [:, 0:16:3, :] (strided with inner rows); c1: [:, :, 1:64] (run); c2: [3, 15::-3, :]
    sel[0][1][1] = 3; sel[0][1][2] = 6;
    sel[1][2][0] = 1; sel[1][2][2] = 63;
    sel[2][0][0] = 3; sel[2][0][2] = 1; sel[2][1][0] = 15; sel[2][1][1] = -3; sel[2][1][2] = 6;
    int32_t *dsel, *dout; uint8_t *ddata;
    (void)hipMalloc(&dsel, sizeof(sel)); (void)hipMalloc(&dout, n * 16 * 4); (void)hipMalloc(&ddata, 1 << 20);
    (void)hipMemcpy(dsel, sel, sizeof(sel), hipMemcpyHostToDevice);
    ReduceArgs a;
    memset(&a, 0, sizeof(a));
    a.data = ddata; a.sel = dsel; a.ndim = 3; a.chunk_elems = 16 * 16 * 64; a.tpc = 1;
    int64_t st = 1;
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        if (d < 3) { a.shape[d] = shape[d]; a.cstride[d] = st; st *= shape[d]; } else { a.shape[d] = 1; a.cstride[d] = 0; }
    }
    hipLaunchKernelGGL(k_dbg, dim3(n), dim3(64), 0, 0, a, dout);
    int32_t h[n * 16];
    (void)hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int c = 0; c < n; ++c) {
        const int32_t *o = h + c * 16;
        printf("chunk %d select: ok %d kk %d m_in %d ext %d istep %d off %d per_span %d | branch: ok %d kk %d m_in %d ext %d "
               "istep %d off %d per_span %d\n", c, o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[8], o[9], o[10], o[11],
               o[12], o[13], o[14]);
        for (int f = 0; f < 7; ++f) bad += o[f] != o[8 + f];
    }
    printf(bad ? "MISMATCH\n" : "branch form == select form\n");
    return bad != 0;
}
