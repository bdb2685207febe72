// colwalk_probe.hip — HBM read-rate probe for the access shapes of the
// partial-axis kernels (not part of the product; tools/README.md).
//
// A 4 GiB buffer laid out like C3: 4096 chunks of 1 MiB (64 rows x 16 KiB),
// chunk (a, b, c) of a 16^3 grid at ((a*16 + b)*16 + c) MiB.  Every kernel
// reads every byte once and sums floats (one v_add per element, so the
// shapes are compared on memory behaviour alone):
//   contig     k_reduce's shape: each block streams whole chunks, 16 KiB per
//              block step (4 loads per lane in flight)
//   col<I,D>   the axis-(0,) column walk: a lane owns I 16-B items of a
//              chunk column (spaced 1 KiB apart, so a wave reads I KiB of a
//              row), walks the 64 rows x 16 layers, D groups of 4 rows in
//              flight
// Build: hipcc -O3 --offload-arch=gfx950 tools/colwalk_probe.hip -o colwalk_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int64_t kChunk = 1 << 20, kRow = 16 << 10, kRows = 64, kGrid = 16;
constexpr int64_t kTotal = kChunk * kGrid * kGrid * kGrid;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt(const uint4 *p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ float sum4(uint4 v) {
    return __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w);
}

// contiguous: block b streams chunks b, b + grid, ...; 256 threads x 4 x 16 B per step
__global__ __launch_bounds__(256) void k_contig(const uint4 *buf, float *out, int64_t nchunks) {
    float acc = 0.f;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint4 *p = buf + c * (kChunk / 16);
        uint4 cur[4], nxt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = ldnt(p + threadIdx.x + u * 256);
        for (int s = 1; s < kChunk / 16 / 1024; ++s) {
#pragma unroll
            for (int u = 0; u < 4; ++u) nxt[u] = ldnt(p + s * 1024 + threadIdx.x + u * 256);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += sum4(cur[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += sum4(cur[u]);
    }
    if (acc == 1.2345f) out[0] = acc;   // keep the loads
}

// column walk: grid = 256 columns (b, c) x blocks per column x L layer
// ranges; block j of a column owns items [j*256*I, (j+1)*256*I) of the 1024
// items of a row, wave w the stripe of 64*I items from j*256*I + 64*I*w, and
// lane t items stripe + t + 64*k, k < I (a wave reads I KiB of a row per
// row step); the block walks 16/L layers
template <int I, int D, int L>
__global__ __launch_bounds__(256) void k_col(const uint4 *buf, float *out) {
    constexpr int bpc = 1024 / (256 * I);
    const int lr = blockIdx.x % L, bx = blockIdx.x / L;
    const int col = bx / bpc, j = bx - col * bpc;
    const int b = col / kGrid, c = col - b * kGrid;
    const int wave = threadIdx.x / 64, lane = threadIdx.x & 63;
    const int64_t item0 = (int64_t)j * 256 * I + wave * 64 * I + lane;   // + 64*k, k < I
    float acc[I];
#pragma unroll
    for (int k = 0; k < I; ++k) acc[k] = 0.f;
    constexpr int64_t groups = 16 / L * kRows / 4;   // layers x rows / 4
    auto addr = [&](int64_t g, int u, int k) {
        const int64_t a0 = g / (kRows / 4), r = (g - a0 * (kRows / 4)) * 4 + u;
        const int64_t a = lr * (16 / L) + a0;
        const int64_t chunk = (a * kGrid + b) * kGrid + c;
        return buf + chunk * (kChunk / 16) + r * (kRow / 16) + item0 + 64 * k;
    };
    uint4 ring[D][4][I];
#pragma unroll
    for (int s = 0; s < D; ++s)
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < I; ++k) ring[s][u][k] = ldnt(addr(s, u, k));
    for (int64_t g = 0; g < groups; g += D) {
#pragma unroll
        for (int s = 0; s < D; ++s) {
            uint4 cur[4][I];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < I; ++k) cur[u][k] = ring[s][u][k];
            if (g + s + D < groups) {
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < I; ++k) ring[s][u][k] = ldnt(addr(g + s + D, u, k));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < I; ++k) acc[k] += sum4(cur[u][k]);
        }
    }
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < I; ++k) t += acc[k];
    if (t == 1.2345f) out[0] = t;
}

template <typename F>
static float time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9f, tot = 0.f;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tot += ms;
        if (ms < best) best = ms;
    }
    return tot / reps;
}

int main() {
    uint4 *buf;
    float *out;
    CK(hipMalloc(&buf, kTotal));
    CK(hipMalloc(&out, 16));
    CK(hipMemset(buf, 0, kTotal));
    const int reps = 20;
    auto report = [&](const char *name, float ms) {
        printf("{\"shape\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, kTotal / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    for (int blocks : {1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "contig grid %d", blocks);
        report(nm, time_ms([&] { hipLaunchKernelGGL(k_contig, dim3(blocks), dim3(256), 0, 0, buf, out, 4096); }, reps));
    }
    // SH: dynamic LDS per block, 40 KiB caps residency at 4 blocks (16 waves) per CU
#define COL(I, D, L, SH) report("col I" #I " D" #D " L" #L " lds" #SH, time_ms([&] { \
        hipLaunchKernelGGL((k_col<I, D, L>), dim3(256 * (4 / I) * L), dim3(256), SH, 0, buf, out); }, reps))
    COL(1, 1, 1, 0); COL(1, 2, 1, 0); COL(1, 3, 1, 0); COL(1, 2, 2, 0); COL(1, 2, 4, 0);
    COL(2, 1, 2, 0); COL(2, 2, 2, 0); COL(2, 1, 4, 0);
    COL(4, 1, 4, 0); COL(4, 2, 4, 0); COL(4, 1, 8, 0);
    // fewer waves with more contiguity; more waves at capped residency
    COL(2, 1, 1, 0); COL(2, 2, 1, 0); COL(4, 1, 1, 0); COL(4, 1, 2, 0);
    COL(1, 2, 2, 40960); COL(2, 1, 2, 40960); COL(4, 1, 4, 40960); COL(2, 1, 4, 40960);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
