// Round 6: span_plan's branch form and select form
// (pyas_kernels.hpp) restated as host C++ and run under UBSan on the three
// selections of span_plan_dbg.hip: undefined behaviour in the source (a
// shift past the width, a signed overflow, an out-of-bounds index) would
// abort here.  The structs carry the fields span_plan reads.
#include <cstdint>
#include <cstdio>
#include <cstring>

constexpr int kMaxDims = 8, kBlock = 256;
struct Sel { int32_t start[kMaxDims], step[kMaxDims], cnt[kMaxDims]; };
struct Args {
    int ndim;
    int64_t shape[kMaxDims], cstride[kMaxDims], chunk_elems;
    bool tab_on[2];
    const int32_t *pool;
};
struct Plan { int kk; int32_t m_in, ext, istep, off, G, P; int64_t nspans, per_span; };

static int64_t sel_index(const Sel &s, const int32_t *pool, int d, int64_t k) {
    return s.step[d] != 0 ? (int64_t)s.start[d] + k * s.step[d] : (int64_t)pool[s.start[d] + k];
}

template <bool BRANCH>
static bool span_plan(const Args &a, uintptr_t base, const Sel &s, Plan &sp) {
    constexpr int ES = 4, NU = 16 / ES;   // float, unshuffled
    if (a.tab_on[0] || a.tab_on[1] || a.chunk_elems >= (int64_t(1) << 31)) return false;
    int k = -1;
    for (int d = kMaxDims - 1; d >= 0; --d)
        if (d < a.ndim && k < 0 && !(s.step[d] == 1 && s.start[d] == 0 && (int64_t)s.cnt[d] == a.shape[d])) k = d;
    if (k < 0) return false;
    int64_t cs_k = 1, sk = 1, st_k = 0, cn_k = 1;
    for (int d = 0; d < kMaxDims; ++d)
        if (d == k) { cs_k = a.cstride[d]; sk = s.step[d]; st_k = s.start[d]; cn_k = s.cnt[d]; }
    if (sk < 0) { st_k += (cn_k - 1) * sk; sk = -sk; }
    const bool run = sk == 1 && (cn_k * cs_k + NU - 1) / NU + 1 <= kBlock;
    const bool strided = !run && sk > 1 && k == a.ndim - 1;
    if (BRANCH) {
        if (run) { sp.kk = k; sp.m_in = (int32_t)(st_k * cs_k); sp.ext = (int32_t)(cn_k * cs_k); sp.istep = 1; sp.per_span = cn_k * cs_k; }
        else if (strided) { sp.kk = k; sp.m_in = (int32_t)st_k; sp.ext = (int32_t)((cn_k - 1) * sk + 1); sp.istep = (int32_t)sk; sp.per_span = cn_k; }
        else { sp.kk = k + 1; sp.m_in = 0; sp.ext = (int32_t)cs_k; sp.istep = 1; sp.per_span = cs_k; }
    } else {
        sp.kk = (run || strided) ? k : k + 1;
        const int64_t m_in = run ? st_k * cs_k : strided ? st_k : 0;
        const int64_t ext = run ? cn_k * cs_k : strided ? (cn_k - 1) * sk + 1 : cs_k;
        sp.m_in = (int32_t)m_in;
        sp.ext = (int32_t)ext;
        sp.istep = strided ? (int32_t)sk : 1;
        sp.per_span = run ? cn_k * cs_k : strided ? cn_k : cs_k;
    }
    int64_t m0 = sp.m_in, nsp = 1;
    for (int d = 0; d < kMaxDims; ++d) {
        if (d < sp.kk) {
            nsp *= s.cnt[d];
            if (s.cnt[d] > 0) m0 += sel_index(s, a.pool, d, 0) * a.cstride[d];
            if (s.cnt[d] > 1) {
                if (s.step[d] == 0 && d < sp.kk - 1) return false;
                const int64_t delta = (s.step[d] != 0 ? (int64_t)s.step[d] : 1) * a.cstride[d];
                if (((delta * ES) & 15) != 0) return false;
            }
        }
    }
    sp.nspans = nsp;
    sp.off = (int32_t)(((base + (uint64_t)(m0 * ES)) & 15) / ES);
    const int64_t G = (sp.off + (int64_t)sp.ext + NU - 1) / NU;
    if (G < 1 || G > kBlock) return false;
    sp.G = (int32_t)G;
    sp.P = (int32_t)(kBlock / G);
    return true;
}

int main() {
    Args a;
    std::memset(&a, 0, sizeof(a));
    a.ndim = 3;
    const int64_t shape[3] = {16, 16, 64};
    int64_t st = 1;
    for (int d = kMaxDims - 1; d >= 0; --d) {
        a.shape[d] = d < 3 ? shape[d] : 1;
        a.cstride[d] = d < 3 ? st : 0;
        if (d < 3) st *= shape[d];
    }
    a.chunk_elems = 16 * 16 * 64;
    Sel s[3];
    for (auto &x : s)
        for (int d = 0; d < kMaxDims; ++d) { x.start[d] = 0; x.step[d] = 1; x.cnt[d] = d < 3 ? (int32_t)shape[d] : 1; }
    s[0].step[1] = 3; s[0].cnt[1] = 6;
    s[1].start[2] = 1; s[1].cnt[2] = 63;
    s[2].start[0] = 3; s[2].cnt[0] = 1; s[2].start[1] = 15; s[2].step[1] = -3; s[2].cnt[1] = 6;
    int bad = 0;
    for (int c = 0; c < 3; ++c) {
        Plan p, q;
        std::memset(&p, 0, sizeof(p));
        std::memset(&q, 0, sizeof(q));
        const bool okp = span_plan<false>(a, 0x1000, s[c], p), okq = span_plan<true>(a, 0x1000, s[c], q);
        std::printf("chunk %d select: ok %d kk %d m_in %d ext %d istep %d off %d per_span %lld | branch: ok %d kk %d m_in %d "
                    "ext %d istep %d off %d per_span %lld\n", c, okp, p.kk, p.m_in, p.ext, p.istep, p.off,
                    (long long)p.per_span, okq, q.kk, q.m_in, q.ext, q.istep, q.off, (long long)q.per_span);
        bad += okp != okq || std::memcmp(&p, &q, sizeof(p)) != 0;
    }
    std::printf(bad ? "MISMATCH\n" : "host: branch form == select form, no UB reported\n");
    return bad != 0;
}
