// debug: evaluate span_plan on the device for a few selections
#include "../../pyactivestorage_amd/csrc/pyas_kernels.hpp"
#include <cstdio>
#include <cstring>
using namespace pyas;
__global__ void k_dbg(ReduceArgs a, int32_t *out) {
    Sel s;
    load_sel(s, a.sel, blockIdx.x, a.ndim, a.shape);
    SpanPlan sp;
    const bool ok = span_plan<float, false>(a, a.data, s, sp);
    if (threadIdx.x == 0) {
        int32_t *o = out + blockIdx.x * 12;
        o[0] = ok; o[1] = sp.kk; o[2] = sp.m_in; o[3] = sp.ext; o[4] = sp.istep; o[5] = sp.off;
        o[6] = sp.G; o[7] = sp.P; o[8] = (int32_t)sp.nspans; o[9] = (int32_t)sp.per_span;
    }
}
int main() {
    const int n = 3;
    int32_t sel[n][PYAS_MAX_DIMS][3];
    for (int c = 0; c < n; ++c)
        for (int d = 0; d < PYAS_MAX_DIMS; ++d) { sel[c][d][0] = 0; sel[c][d][1] = 1; sel[c][d][2] = 1; }
    int64_t shape[3] = {16, 16, 64};
    // c0: [:, 0:16:3, :]; c1: [:, :, 1:64]; c2: [3, 15::-3, :]
    for (int c = 0; c < n; ++c) for (int d = 0; d < 3; ++d) { sel[c][d][0] = 0; sel[c][d][1] = 1; sel[c][d][2] = (int)shape[d]; }
    sel[0][1][1] = 3; sel[0][1][2] = 6;
    sel[1][2][0] = 1; sel[1][2][2] = 63;
    sel[2][0][0] = 3; sel[2][0][2] = 1; sel[2][1][0] = 15; sel[2][1][1] = -3; sel[2][1][2] = 6;
    int32_t *dsel, *dout; uint8_t *ddata;
    hipMalloc(&dsel, sizeof(sel)); hipMalloc(&dout, n * 12 * 4); hipMalloc(&ddata, 1 << 20);
    hipMemcpy(dsel, sel, sizeof(sel), hipMemcpyHostToDevice);
    ReduceArgs a; memset(&a, 0, sizeof(a));
    a.data = ddata; a.sel = dsel; a.ndim = 3; a.chunk_elems = 16 * 16 * 64; a.tpc = 1;
    int64_t st = 1;
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        if (d < 3) { a.shape[d] = shape[d]; a.cstride[d] = st; st *= shape[d]; } else { a.shape[d] = 1; a.cstride[d] = 0; }
    }
    hipLaunchKernelGGL(k_dbg, dim3(n), dim3(256), 0, 0, a, dout);
    int32_t h[n * 12];
    hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
    for (int c = 0; c < n; ++c) {
        printf("chunk %d: ok %d kk %d m_in %d ext %d istep %d off %d G %d P %d nspans %d per_span %d\n", c, h[c*12], h[c*12+1],
               h[c*12+2], h[c*12+3], h[c*12+4], h[c*12+5], h[c*12+6], h[c*12+7], h[c*12+8], h[c*12+9]);
    }
    return 0;
}
