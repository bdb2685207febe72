// pyas_inflate.hip — zlib (RFC 1950) / DEFLATE (RFC 1951) decoding on gfx950.
//
// Row f3 of the hot-path table: the reference inflates every compressed chunk
// on the host, `numcodecs.Zlib.decode` -> `zlib.decompress` (built at
// activestorage/hdf2numcodec.py:34-35, applied at activestorage/storage.py:
// 119-120).  Here one wave64 inflates one chunk stream; a launch covers every
// chunk of a query, so thousands of streams decode concurrently.
//
// Per wave:
//   * input: a 128-dword LDS ring refilled 64 dwords at a time from a block
//     loaded one refill ahead, so the window's bits are two LDS dwords per
//     lane and the symbol loop never waits on a global load;
//   * Huffman decode: 10-bit literal/length and 8-bit distance lookup tables
//     in LDS, canonical walk for longer codes;
//   * symbols: a speculative window -- every lane decodes the symbol that
//     would start at its bit offset, one v_readlane per symbol walks the real
//     chain, and the window's output bytes are produced lane-parallel (one
//     lane per output byte, matches resolved by pointer jumping);
//   * output: the most recent 2^WBITS bytes (8-32 KiB) live in an LDS ring,
//     flushed to HBM in coalesced 1 KiB pieces with Adler-32 folded in per
//     flush by a wave reduction;
//   * a match reaching further back than the ring (d > 2^WBITS, up to
//     DEFLATE's 32 KiB) reads the already-flushed output from HBM after the
//     wave's stores have drained, with L1-bypassing (agent-scope) loads.
//     A smaller ring is what buys occupancy: 2^13 B + tables ~= 12.7 KiB of
//     LDS per wave -> 12 streams per CU instead of 4.
// Error behaviour follows zlib's inflate(): bad header, preset dictionary,
// invalid block type, stored-length mismatch, over-subscribed or incomplete
// codes, invalid symbols, distance too far back, truncated input and Adler-32
// mismatch are all reported per stream (pyas_inflate_status in pyas.h).
#include "pyas_internal.hpp"

namespace pyas {
namespace {

constexpr int kLitBits = 10, kDistBits = 8;

constexpr uint32_t kFlush = 1024;   // bytes per coalesced flush (16 per lane)

__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                        2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                         33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                         1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                         6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Code tables + build scratch (the history window is separate: its size is a
// template parameter of the kernel).
struct Lds {
    uint16_t lit[1 << kLitBits];    // sym | len << 9; len 0 -> canonical walk
    uint16_t dist[1 << kDistBits];
    uint16_t lit_cnt[16], dist_cnt[16];
    uint16_t lit_sym[288], dist_sym[32];
    uint16_t code[320];             // canonical code per symbol (build scratch)
    uint16_t offs[16], next[16];    // build scratch
    uint8_t lens[320];              // code lengths: literal/length then distance
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Bit reader over dword-aligned input, staged through a 128-dword LDS ring:
// the wave's window bits come from two LDS dwords per lane (no readlanes, no
// vector-memory wait in the symbol loop).  The ring is refilled 64 dwords at
// a time from a block loaded into one VGPR per lane a refill earlier, so the
// global load latency is off the decode path.
constexpr uint32_t kInRing = 128, kInBlock = 64;

struct BitIn {
    const uint32_t *w;
    uint32_t nwords;   // readable dwords from w
    uint32_t nbits;    // valid bits from w (stream end)
    uint32_t pos;      // bit position from w
    uint32_t filled;   // dwords [filled - kInRing, filled) are in the ring
    uint32_t stage;    // w[filled + lane], loaded ahead
    uint32_t *ring;    // LDS

    __device__ __forceinline__ uint32_t load(uint32_t k) const {
        const uint32_t i = k + (threadIdx.x & 63);
        return i < nwords ? __builtin_nontemporal_load(w + i) : 0u;
    }
    __device__ __forceinline__ void seek() {   // at the start and after stored blocks
        filled = pos >> 5;
        ring[(filled + (threadIdx.x & 63)) & (kInRing - 1)] = load(filled);
        filled += kInBlock;
        stage = load(filled);
    }
    __device__ __forceinline__ void ensure() {
        if ((pos >> 5) + 32u > filled) {
            ring[(filled + (threadIdx.x & 63)) & (kInRing - 1)] = stage;
            filled += kInBlock;
            stage = load(filled);
        }
    }
    // 32 bits at pos + off (LSB first), per lane
    __device__ __forceinline__ uint32_t bits_at(uint32_t off) const {
        const uint32_t t = pos + off, k = t >> 5;
        return __builtin_amdgcn_alignbit(ring[(k + 1) & (kInRing - 1)], ring[k & (kInRing - 1)], t & 31);
    }
    // At least 32 valid bits starting at pos (uniform).
    __device__ __forceinline__ uint32_t peek() {
        ensure();
        return uni(bits_at(0));
    }
};

// Canonical Huffman table for `n` code lengths in L.lens[first..first+n).
// Returns 0, or PYAS_INFLATE_BAD_CODE for over-subscribed / disallowed
// incomplete sets (zlib inflate_table rules: incomplete only for a single
// length-1 code in the literal/length and distance trees).
__device__ int build(Lds &L, int first, int n, uint16_t *cnt, uint16_t *sorted, uint16_t *tab, int P,
                     bool code_lengths) {
    const int lane = threadIdx.x & 63;
    for (int k = lane; k < (1 << P); k += 64) tab[k] = 0;
    __shared__ int s_status;
    if (lane == 0) {
        for (int l = 0; l < 16; ++l) cnt[l] = 0;
        for (int s = 0; s < n; ++s) cnt[L.lens[first + s]]++;
        cnt[0] = 0;
        int max = 0;
        for (int l = 1; l < 16; ++l)
            if (cnt[l]) max = l;
        int left = 1, status = 0;
        for (int l = 1; l < 16; ++l) {
            left = (left << 1) - cnt[l];
            if (left < 0) status = PYAS_INFLATE_BAD_CODE;
        }
        if (left > 0 && max > 0 && (code_lengths || max != 1)) status = PYAS_INFLATE_BAD_CODE;
        uint16_t *offs = L.offs, *next = L.next;
        offs[1] = 0;
        next[1] = 0;
        for (int l = 1; l < 15; ++l) {
            offs[l + 1] = offs[l] + cnt[l];
            next[l + 1] = (uint16_t)((next[l] + cnt[l]) << 1);
        }
        for (int s = 0; s < n; ++s) {
            const int l = L.lens[first + s];
            if (l) {
                sorted[offs[l]++] = (uint16_t)s;
                L.code[s] = next[l]++;
            }
        }
        s_status = status;
    }
    __syncthreads();
    for (int s = lane; s < n; s += 64) {
        const int l = L.lens[first + s];
        if (l && l <= P) {
            const uint32_t rc = __builtin_bitreverse32((uint32_t)L.code[s]) >> (32 - l);
            const uint16_t e = (uint16_t)(s | (l << 9));
            for (uint32_t k = rc; k < (1u << P); k += 1u << l) tab[k] = e;
        }
    }
    __syncthreads();
    return uni((uint32_t)s_status);
}

// Decode one symbol: table hit, else canonical walk over the peeked bits.
// Returns sym and sets len (0 on an invalid code).
__device__ __forceinline__ uint32_t decode(uint32_t bits, const uint16_t *tab, int P, const uint16_t *cnt,
                                           const uint16_t *sorted, uint32_t &len) {
    const uint32_t e = uni(tab[bits & ((1u << P) - 1)]);
    if (e >> 9) {
        len = e >> 9;
        return e & 511u;
    }
    int code = 0, firstc = 0, index = 0;
    for (int l = 1; l < 16; ++l) {
        code |= (bits >> (l - 1)) & 1u;
        const int count = cnt[l];
        if (code - firstc < count) {
            len = (uint32_t)l;
            return uni(sorted[index + code - firstc]);
        }
        index += count;
        firstc = (firstc + count) << 1;
        code <<= 1;
    }
    len = 0;
    return 0;
}

struct Out {
    uint8_t *dst;
    uint32_t cap, pos, fpos;
    uint32_t a, b;   // Adler-32 state
    bool aligned;
};

// Write ring bytes [fpos, fpos + n) to dst, folding them into Adler-32.
template <uint32_t MASK>
__device__ void flush(const uint8_t *win, Out &o, uint32_t n) {
    const int lane = threadIdx.x & 63;
    uint32_t s = 0, t = 0;
    if (n == kFlush && o.aligned) {   // 16 bytes per lane, 1 KiB coalesced
        const uint32_t off = o.fpos + lane * 16;
        const uint4 v = *reinterpret_cast<const uint4 *>(&win[off & MASK]);
        *reinterpret_cast<uint4 *>(o.dst + off) = v;
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t byte = (w4[k >> 2] >> ((k & 3) * 8)) & 255u;
            s += byte;
            t += (n - (lane * 16 + k)) * byte;
        }
    } else {
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t byte = win[(o.fpos + i) & MASK];
            o.dst[o.fpos + i] = (uint8_t)byte;
            s += byte;
            t += (n - i) * byte;
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        s += (uint32_t)__shfl_xor((int)s, m, 64);
        t += (uint32_t)__shfl_xor((int)t, m, 64);
    }
    s = uni(s);
    t = uni(t);
    // a' = a + sum b_i;  b' = b + n*a + sum (n - i) b_i   (mod 65521)
    const uint64_t bb = (uint64_t)o.b + (uint64_t)n * o.a + t;
    o.a = (o.a + s) % 65521u;
    o.b = (uint32_t)(bb % 65521u);
    o.fpos += n;
}

}  // namespace

// Inclusive prefix sum over the wave: DPP shifts inside each 16-lane row,
// then the row totals (lanes 15, 31, 47) added with three readlanes.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    const int lane = threadIdx.x & 63;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
    const uint32_t row = (uint32_t)lane >> 4;
    return x + (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
}

// LDS written by other lanes of this wave is read after this point (the
// compiler may not forward a lane's own earlier store across it).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    const int lane = threadIdx.x & 63;
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true));
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
    const uint32_t row = (uint32_t)lane >> 4;
    uint32_t c = row >= 1 ? r0 : 0u;
    c = row >= 2 ? max(c, r1) : c;
    c = row >= 3 ? max(c, r2) : c;
    return max(x, c);
}

// Byte of already-flushed output, coherent with this wave's earlier stores.
__device__ __forceinline__ uint32_t far_byte(const uint8_t *p) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (v >> (((uintptr_t)p & 3) * 8)) & 255u;
}

// Phase timing (diagnostic build, -DPYAS_INFLATE_PROF): per-wave cycle sums
// of the decode phases, printed for the first streams of a launch.
#ifdef PYAS_INFLATE_PROF
#define PYAS_PROF_INIT uint64_t pf_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}; uint64_t pf_last = clock64(); \
                       uint64_t pf_st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PYAS_STAT(i, v) (pf_st[i] += (v))
#define PYAS_PROF(i) do { const uint64_t pf_n = clock64(); pf_acc[i] += pf_n - pf_last; pf_last = pf_n; \
                          if ((i) == 0) pf_acc[8]++; } while (0)
#else
#define PYAS_PROF_INIT
#define PYAS_PROF(i) do { } while (0)
#define PYAS_STAT(i, v) ((void)0)
#endif

template <int WBITS>
__global__ __launch_bounds__(64) void k_inflate(InflateArgs x) {
    PYAS_PROF_INIT
    constexpr uint32_t kWin = 1u << WBITS, kWinMask = kWin - 1;
    static_assert(kWin >= 4096, "ring must exceed the unflushed bytes plus one match");
    __shared__ Lds L;
    __shared__ alignas(16) uint8_t win[kWin];
    const int64_t c = blockIdx.x;
    const int lane = threadIdx.x;
    const uint8_t *src = x.src + x.src_offsets[c];
    const int64_t n_in = x.src_sizes[c];
    const uint32_t mis = (uint32_t)((uintptr_t)src & 3);
    __shared__ uint32_t in_ring[kInRing];
    __shared__ uint8_t mark[64];              // symbol starts of one 64-byte output step
    BitIn in;
    in.ring = in_ring;
    in.w = reinterpret_cast<const uint32_t *>(src - mis);
    in.nbits = (uint32_t)((n_in + mis) * 8);
    in.nwords = (uint32_t)((n_in + mis + 3) / 4);
    in.pos = mis * 8;
    in.seek();
    Out o;
    o.dst = x.dst + x.dst_offsets[c];
    o.cap = (uint32_t)x.dst_capacity[c];
    o.pos = o.fpos = 0;
    o.a = 1;
    o.b = 0;
    o.aligned = (((uintptr_t)o.dst) & 15) == 0;
    int status = PYAS_INFLATE_OK;

    // zlib header (RFC 1950): CM 8, CINFO <= 7, FCHECK, no preset dictionary
    if (n_in < 6) status = PYAS_INFLATE_TRUNCATED;
    if (status == 0) {
        const uint32_t h = in.peek();
        const uint32_t cmf = h & 255u, flg = (h >> 8) & 255u;
        if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u)
            status = PYAS_INFLATE_BAD_HEADER;
        else if (flg & 32u)
            status = PYAS_INFLATE_NEED_DICT;
        in.pos += 16;
    }
    bool last = false;
    while (status == 0 && !last) {
        uint32_t h = in.peek();
        last = h & 1u;
        const uint32_t type = (h >> 1) & 3u;
        in.pos += 3;
        if (type == 0) {   // stored
            in.pos = (in.pos + 7) & ~7u;
            h = in.peek();
            const uint32_t len = h & 0xffffu, nlen = h >> 16;
            in.pos += 32;
            if ((len ^ 0xffffu) != nlen) { status = PYAS_INFLATE_BAD_STORED; break; }
            if (in.pos + len * 8 > in.nbits) { status = PYAS_INFLATE_TRUNCATED; break; }
            if (o.pos + len > o.cap) { status = PYAS_INFLATE_OVERFLOW; break; }
            // 16 bytes per lane per 1 KiB step: five independent dword loads
            // (the stream is dword-aligned at in.w), realigned with alignbyte
            const uint32_t byte0 = in.pos >> 3;
            for (uint32_t done = 0; done < len;) {
                while (o.pos - o.fpos >= kFlush) flush<kWinMask>(win, o, kFlush);
                const uint32_t step = min(len - done, kFlush);
                const uint32_t mine = (uint32_t)lane * 16u;
                if (mine < step) {
                    const uint32_t b = byte0 + done + mine;
                    const uint32_t wi = b >> 2, sh = b & 3u;
                    uint32_t dw[5];
#pragma unroll
                    for (uint32_t k = 0; k < 5; ++k)
                        dw[k] = wi + k < in.nwords ? __builtin_nontemporal_load(in.w + wi + k) : 0u;
                    const uint32_t n = min(step - mine, 16u);
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) {
                        const uint32_t q = __builtin_amdgcn_alignbyte(dw[k + 1], dw[k], sh);
#pragma unroll
                        for (uint32_t m = 0; m < 4; ++m)
                            if (k * 4 + m < n) win[(o.pos + mine + k * 4 + m) & kWinMask] = (uint8_t)(q >> (8 * m));
                    }
                }
                o.pos += step;
                done += step;
                __syncthreads();
            }
            in.pos += len * 8;
            in.seek();
            continue;
        }
        const uint16_t *lit = L.lit, *dist = L.dist;
        if (type == 1) {   // fixed codes (RFC 1951 3.2.6)
            for (int s = lane; s < 320; s += 64)
                L.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
            __syncthreads();
            build(L, 0, 288, L.lit_cnt, L.lit_sym, L.lit, kLitBits, false);
            build(L, 288, 32, L.dist_cnt, L.dist_sym, L.dist, kDistBits, false);
        } else if (type == 2) {   // dynamic codes
            h = in.peek();
            const uint32_t nlen = (h & 31u) + 257, ndist = ((h >> 5) & 31u) + 1, ncode = ((h >> 10) & 15u) + 4;
            in.pos += 14;
            if (nlen > 286 || ndist > 30) { status = PYAS_INFLATE_BAD_CODE; break; }
            // code-length code: 3 bits per length in c_clen_order
            h = in.peek();
            const uint32_t h2 = [&] { in.pos += 30; const uint32_t r = in.peek(); in.pos -= 30; return r; }();
            for (int s = lane; s < 19; s += 64) {
                const uint32_t bit = 3u * (uint32_t)s;
                uint32_t v = 0;
                if ((uint32_t)s < ncode) v = bit < 30 ? (h >> bit) & 7u : (h2 >> (bit - 30)) & 7u;
                L.lens[c_clen_order[s]] = (uint8_t)v;
            }
            in.pos += 3 * ncode;
            __syncthreads();
            // the code-length tree uses the distance table slots (7-bit codes)
            if (build(L, 0, 19, L.dist_cnt, L.dist_sym, L.dist, 7, true)) { status = PYAS_INFLATE_BAD_CODE; break; }
            // code lengths for literal/length + distance, serial (<= 316)
            uint32_t k = 0;
            uint32_t prev = 0;
            while (k < nlen + ndist) {
                const uint32_t bits = in.peek();
                uint32_t l;
                const uint32_t sym = decode(bits, L.dist, 7, L.dist_cnt, L.dist_sym, l);
                if (!l) { status = PYAS_INFLATE_BAD_CODE; break; }
                in.pos += l;
                const uint32_t more = bits >> l;
                uint32_t rep, val;
                if (sym < 16) {
                    rep = 1; val = sym; prev = sym;
                } else if (sym == 16) {
                    if (k == 0) { status = PYAS_INFLATE_BAD_CODE; break; }
                    rep = 3 + (more & 3u); val = prev; in.pos += 2;
                } else if (sym == 17) {
                    rep = 3 + (more & 7u); val = 0; in.pos += 3;
                } else {
                    rep = 11 + (more & 127u); val = 0; in.pos += 7;
                }
                if (k + rep > nlen + ndist) { status = PYAS_INFLATE_BAD_CODE; break; }
                if (sym > 16) prev = 0;   // zlib: repeat-previous after zeros repeats zero
                for (uint32_t i = lane; i < rep; i += 64) {
                    const uint32_t s = k + i;
                    L.lens[s < nlen ? s : 288 + (s - nlen)] = (uint8_t)val;
                }
                k += rep;
            }
            if (status) break;
            for (int s = nlen + lane; s < 288; s += 64) L.lens[s] = 0;
            for (int s = 288 + (int)ndist + lane; s < 320; s += 64) L.lens[s] = 0;
            __syncthreads();
            if (L.lens[256] == 0) { status = PYAS_INFLATE_BAD_CODE; break; }
            if (build(L, 0, 288, L.lit_cnt, L.lit_sym, L.lit, kLitBits, false) ||
                build(L, 288, 32, L.dist_cnt, L.dist_sym, L.dist, kDistBits, false)) {
                status = PYAS_INFLATE_BAD_CODE;
                break;
            }
        } else {
            status = PYAS_INFLATE_BAD_BLOCK;
            break;
        }
        // Match copy out[p+i] = out[p-d+(i mod d)], lane-parallel (all
        // sources precede p); beyond the ring every source byte is in dst.
        auto copy_match = [&](uint32_t d, uint32_t len) {
            const uint32_t from = o.pos - d;
            if (d > kWin) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                for (uint32_t r = 0; r < len; r += 64) {
                    const uint32_t i = r + lane;
                    if (i < len) win[(o.pos + i) & kWinMask] = (uint8_t)far_byte(o.dst + from + i);
                }
            } else {
                for (uint32_t r = 0; r < len; r += 64) {
                    const uint32_t i = r + lane;
                    if (i < len) {
                        const uint32_t srcp = from + (d >= len ? i : i % d);
                        win[(o.pos + i) & kWinMask] = win[srcp & kWinMask];
                    }
                }
            }
            o.pos += len;
        };
        // A short match (len <= 64, source in the ring) is split: its ring
        // read is issued at once, its write is deferred until the next ring
        // read or flush, so the LDS round trip overlaps the decode of the
        // symbols that follow (they only write later positions).
        uint32_t pend_v = 0, pend_p = 0, pend_n = 0;
        auto issue_pending = [&]() {
            if (pend_n) {
                if ((uint32_t)lane < pend_n) win[(pend_p + lane) & kWinMask] = (uint8_t)pend_v;
                pend_n = 0;
            }
        };
        auto start_match = [&](uint32_t d, uint32_t len) {
            issue_pending();
            if (len <= 64 && d <= kWin) {
                const uint32_t from = o.pos - d;
                const uint32_t i = (uint32_t)lane < len ? (uint32_t)lane : 0u;
                pend_v = win[(from + (d >= len ? i : i % d)) & kWinMask];
                pend_p = o.pos;
                pend_n = len;
                o.pos += len;
            } else {
                copy_match(d, len);
            }
        };
        // One symbol, any code length (canonical walk past the root tables).
        // Returns 0 = continue, 1 = end of block, 2 = error (status set).
        auto one_symbol = [&]() -> int {
            issue_pending();
            if (o.pos - o.fpos >= kFlush) flush<kWinMask>(win, o, kFlush);
            if (in.pos > in.nbits) { status = PYAS_INFLATE_TRUNCATED; return 2; }
            uint32_t bits = in.peek();
            uint32_t l;
            uint32_t sym = decode(bits, lit, kLitBits, L.lit_cnt, L.lit_sym, l);
            if (!l) { status = PYAS_INFLATE_BAD_SYMBOL; return 2; }
            if (sym < 256) {
                if (o.pos >= o.cap) { status = PYAS_INFLATE_OVERFLOW; return 2; }
                if (lane == 0) win[o.pos & kWinMask] = (uint8_t)sym;
                o.pos++;
                in.pos += l;
                return 0;
            }
            if (sym == 256) { in.pos += l; return 1; }
            sym -= 257;
            if (sym >= 29) { status = PYAS_INFLATE_BAD_SYMBOL; return 2; }
            const uint32_t le = c_len_extra[sym];
            const uint32_t len = c_len_base[sym] + ((bits >> l) & ((1u << le) - 1u));
            in.pos += l + le;
            bits = in.peek();
            const uint32_t ds = decode(bits, dist, kDistBits, L.dist_cnt, L.dist_sym, l);
            if (!l || ds >= 30) { status = PYAS_INFLATE_BAD_SYMBOL; return 2; }
            const uint32_t de = c_dist_extra[ds];
            const uint32_t d = c_dist_base[ds] + ((bits >> l) & ((1u << de) - 1u));
            in.pos += l + de;
            if (d > o.pos) { status = PYAS_INFLATE_BAD_DISTANCE; return 2; }
            if (o.pos + len > o.cap) { status = PYAS_INFLATE_OVERFLOW; return 2; }
            copy_match(d, len);
            return 0;
        };
        // Symbol loop over speculative windows.  Lane k holds the 32 bits
        // at pos + k and looks up both root tables there (one LDS round trip
        // for the whole wave).
        //
        // Parallel walk (the common case): every lane decodes the symbol
        // that WOULD start at its bit offset -- literal, or length plus the
        // distance code read from lane k + l + le -- and its successor
        // offset nxt.  Only the chain of successors from offset 0 is then
        // walked on the scalar unit (one v_readlane per symbol); the chain's
        // output offsets come from one wave prefix sum, its literals are
        // written by their own lanes, and its matches are copied in order
        // (literals between two matches are written before the later match
        // reads the ring, as a serial decoder would).  A lane whose symbol
        // cannot be finished inside the window ends the chain there: a code
        // longer than its root table (one_symbol), end of block, or a
        // distance code past the window (next window).  Anything else
        // unusual -- an invalid symbol, truncated input, a distance before
        // the output start, output past capacity -- sends the whole window
        // to the serial walk below, which reports zlib's error at the right
        // symbol.  At most kBudget output bytes per window keep the ring
        // invariants of the serial decoder (unflushed bytes + window output
        // fit the ring; a match source further back than the ring is
        // already flushed to dst).
        constexpr uint32_t kBudget = kWin / 4;
        bool eob = false;
        uint32_t windows_left = in.nbits + 64u;   // every window consumes input; a stuck walk ends here
        while (!eob) {
            PYAS_PROF(7);
            if (windows_left-- == 0u) { status = PYAS_INFLATE_BAD_SYMBOL; break; }
            while (o.pos - o.fpos >= kFlush) {
                issue_pending();
                flush<kWinMask>(win, o, kFlush);
            }
            PYAS_PROF(5);
            in.ensure();                                 // the ring holds the window
            const uint32_t v = in.bits_at((uint32_t)lane);
            const uint32_t E = lit[v & ((1u << kLitBits) - 1u)];
            const uint32_t D = dist[v & ((1u << kDistBits) - 1u)];
            auto rl = [](uint32_t x, uint32_t k) {
                return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)k);
            };
            PYAS_PROF(0);

            // ---- per-lane speculative symbol -------------------------------
            enum : uint32_t { kLit = 0, kMatch = 1, kStop = 2 };
            enum : uint32_t { rSlow = 1, rEob = 2, rNewWin = 3, rSerial = 4 };
            const uint32_t l = E >> 9;
            const uint32_t sym = E & 511u;
            const uint32_t ls = sym - 257u;              // length symbol index (wraps for < 257)
            const uint32_t le = (ls < 8u || ls == 28u) ? 0u : (ls - 4u) >> 2;
            const uint32_t doff = (uint32_t)lane + l + le;
            const uint32_t dsrc = doff < 64u ? doff : 63u;
            const uint32_t f = (uint32_t)__shfl((int)D, (int)dsrc, 64);
            const uint32_t vd = (uint32_t)__shfl((int)v, (int)dsrc, 64);
            // every lane computes all fields; selects pick the symbol's kind
            const uint32_t dl = f >> 9, ds = f & 511u;
            const uint32_t lec = le < 5u ? le : 5u;
            const uint32_t lbase = ls < 8u ? ls + 3u : ls == 28u ? 258u : ((4u + (ls & 3u)) << lec) + 3u;
            const uint32_t de0 = ds < 4u ? 0u : (ds - 2u) >> 1;
            const uint32_t de = de0 < 13u ? de0 : 13u;
            const uint32_t dbase = ds < 4u ? ds + 1u : ((2u + (ds & 1u)) << de) + 1u;
            const uint32_t mlen = lbase + ((v >> l) & ((1u << lec) - 1u));
            const uint32_t mdist = dbase + ((vd >> dl) & ((1u << de) - 1u));
            const bool trunc = in.pos + (uint32_t)lane > in.nbits;
            const uint32_t why = trunc ? rSerial
                               : !l ? rSlow
                               : sym < 256u ? 0u
                               : sym == 256u ? rEob
                               : ls >= 29u ? rSerial
                               : doff > 63u ? rNewWin
                               : !dl ? rSlow
                               : ds >= 30u ? rSerial : 0u;
            const bool is_lit = why == 0u && sym < 256u;
            const uint32_t kind = why ? kStop : is_lit ? kLit : kMatch;
            const uint32_t olen = why ? 0u : is_lit ? 1u : mlen;
            const uint32_t dd = mdist;
            uint32_t nxt = is_lit ? (uint32_t)lane + l : doff + dl + de;
            if (kind == kStop) nxt = 128u + why;         // >= 128: the chain stops here
            PYAS_PROF(1);

            // ---- the chain from offset 0 (scalar) --------------------------
            uint64_t M = 0;
            uint32_t off = 0, prev = 0, stop = 0;
            do {
                M |= 1ull << off;
                prev = off;
                off = rl(nxt, off);
            } while (off < 64u);
            if (off >= 128u) {                           // ended on a stop lane: not consumed
                stop = off - 128u;
                off = prev;
                M &= ~(1ull << prev);
            }
            PYAS_PROF(2);
            const bool on = (M >> lane) & 1ull;
            const uint32_t incl = wave_incl_sum(on ? olen : 0u);   // output bytes up to this lane
            const uint32_t excl = incl - (on ? olen : 0u);
            uint32_t T = rl(incl, 63);
            bool par = stop != rSerial || off > 0;
            if (par && T > kBudget) {                    // end the window before the first symbol past it
                const uint64_t over = __ballot(on && incl > kBudget);
                const uint32_t cut = (uint32_t)__builtin_ctzll(over);
                M &= (1ull << cut) - 1ull;
                off = cut;
                stop = 0;
                T = rl(excl, cut);
            }
            const bool on2 = (M >> lane) & 1ull;
            if (par) {
                if (o.pos + T > o.cap) par = false;
                if (__ballot(on2 && kind == kMatch && dd > o.pos + excl)) par = false;
            }
            PYAS_PROF(3);
            if (par) {
                issue_pending();
                const uint32_t pos0 = o.pos;
                uint64_t mm = __ballot(on2 && kind == kMatch);
                PYAS_STAT(0, __builtin_popcountll(M));
                PYAS_STAT(1, __builtin_popcountll(mm));
                PYAS_STAT(2, __builtin_popcountll(__ballot(on2 && kind == kMatch && olen > 64u)));
                PYAS_STAT(3, __builtin_popcountll(__ballot(on2 && kind == kMatch && dd < olen)));
                PYAS_STAT(4, __builtin_popcountll(__ballot(on2 && kind == kMatch && dd < excl + 1u)));
                PYAS_STAT(5, stop == rSlow ? 1u : 0u);
                PYAS_STAT(6, T);
                PYAS_STAT(7, __builtin_popcountll(__ballot(on2 && kind == kMatch && dd > kWin)));
                (void)mm;
                // The window's output, 64 positions per step, one per lane.
                // Lane j takes position p = c + j: the symbol covering p is
                // the last one starting at or before p (start marks in LDS,
                // then a max scan).  A literal gives its byte.  A match byte
                // p copies byte p - d: from the ring when p - d precedes this
                // step (from dst when d exceeds the ring: those bytes are
                // flushed), else from the lane producing p - d in this step;
                // pointer jumping over those lanes ends at a lane whose byte
                // is known (an overlapping match, d < len, chains this way).
                const bool any_far = __ballot(on2 && kind == kMatch && dd > kWin) != 0;
                if (any_far) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t pk = (kind << 16) | (sym & 255u);
                uint32_t carry = 0;                      // lane + 1 of the symbol covering position c
                for (uint32_t c = 0; c < T; c += 64) {
                    const uint32_t p = c + (uint32_t)lane;
                    mark[lane] = 0;
                    if (on2 && excl >= c && excl < c + 64u) mark[excl - c] = (uint8_t)(lane + 1);
                    wave_lds_sync();                     // other lanes' marks (no store forwarding)
                    uint32_t S = wave_incl_max(mark[lane]);
                    S = S > carry ? S : carry;
                    carry = rl(S, 63);
                    const uint32_t k = (S - 1u) & 63u;
                    const uint32_t s_d = (uint32_t)__shfl((int)dd, (int)k, 64);
                    const uint32_t s_pk = (uint32_t)__shfl((int)pk, (int)k, 64);
                    const bool valid = p < T;
                    const bool is_m = (s_pk >> 16) == kMatch;
                    const int32_t src = (int32_t)p - (int32_t)s_d;   // window-relative source
                    const bool inner = is_m && src >= (int32_t)c;
                    uint32_t val = s_pk & 255u;
                    if (valid && is_m && !inner)
                        val = s_d > kWin ? far_byte(o.dst + (pos0 + src)) : (uint32_t)win[(pos0 + src) & kWinMask];
                    if (__ballot(valid && inner)) {
                        // pd = lane whose byte this lane copies | 64 once that
                        // lane's byte is known (a root); undone lanes jump
                        // to their target's pd until every lane has a root
                        uint32_t pd = inner ? (uint32_t)(src - (int32_t)c) : ((uint32_t)lane | 64u);
                        while (__ballot(!(pd & 64u))) {
                            const uint32_t q = (uint32_t)__shfl((int)pd, (int)(pd & 63u), 64);
                            if (!(pd & 64u)) pd = q;
                        }
                        val = (uint32_t)__shfl((int)val, (int)(pd & 63u), 64);
                    }
                    if (valid) win[(pos0 + p) & kWinMask] = (uint8_t)val;
                    wave_lds_sync();
                }
                o.pos = pos0 + T;
                in.pos += off;
                if (stop == rEob) {
                    in.pos += rl(l, off);
                    eob = true;
                } else if (stop == rSlow) {
                    const int r = one_symbol();
                    if (r == 2) break;
                    if (r == 1) eob = true;
                }
                // rNewWin / rSerial past offset 0 / budget cut: next window
                PYAS_PROF(4);
                continue;
            }

            // ---- serial walk of the same window ----------------------------
            off = 0;
            bool slow = false;
            for (;;) {
                if (o.pos - o.fpos >= kFlush) {
                    issue_pending();
                    flush<kWinMask>(win, o, kFlush);
                }
                if (off > 63) break;
                if (in.pos + off > in.nbits) { status = PYAS_INFLATE_TRUNCATED; break; }
                const uint32_t e = rl(E, off);
                const uint32_t el = e >> 9;
                if (!el) { slow = true; break; }
                uint32_t es = e & 511u;
                if (es < 256) {
                    if (o.pos >= o.cap) { status = PYAS_INFLATE_OVERFLOW; break; }
                    if (lane == 0) win[o.pos & kWinMask] = (uint8_t)es;
                    o.pos++;
                    off += el;
                    continue;
                }
                if (es == 256) { off += el; eob = true; break; }
                es -= 257;
                if (es >= 29) { status = PYAS_INFLATE_BAD_SYMBOL; break; }
                const uint32_t sle = (es < 8 || es == 28) ? 0u : (es - 4u) >> 2;
                const uint32_t lbase = es < 8 ? es + 3u : es == 28 ? 258u : ((4u + (es & 3u)) << sle) + 3u;
                const uint32_t sdoff = off + el + sle;
                if (sdoff > 63) break;                   // next window starts at this symbol
                const uint32_t len = lbase + ((rl(v, off) >> el) & ((1u << sle) - 1u));
                const uint32_t sf = rl(D, sdoff);
                const uint32_t dl = sf >> 9;
                if (!dl) { slow = true; break; }         // long distance code
                const uint32_t ds = sf & 511u;
                if (ds >= 30) { status = PYAS_INFLATE_BAD_SYMBOL; break; }
                const uint32_t de = ds < 4 ? 0u : (ds - 2u) >> 1;
                const uint32_t dbase = ds < 4 ? ds + 1u : ((2u + (ds & 1u)) << de) + 1u;
                const uint32_t d = dbase + ((rl(v, sdoff) >> dl) & ((1u << de) - 1u));
                if (d > o.pos) { status = PYAS_INFLATE_BAD_DISTANCE; break; }
                if (o.pos + len > o.cap) { status = PYAS_INFLATE_OVERFLOW; break; }
                off = sdoff + dl + de;
                start_match(d, len);
            }
            if (status) break;
            in.pos += off;
            if (eob) break;
            if (slow) {
                const int r = one_symbol();
                if (r == 2) break;
                if (r == 1) eob = true;
            }
            PYAS_PROF(6);
        }
        issue_pending();
        if (status) break;
    }
    if (status == 0) {
        __syncthreads();
        while (o.pos - o.fpos >= kFlush) flush<kWinMask>(win, o, kFlush);
        if (o.pos > o.fpos) flush<kWinMask>(win, o, o.pos - o.fpos);
        in.pos = (in.pos + 7) & ~7u;
        if (in.pos + 32 > in.nbits) {
            status = PYAS_INFLATE_TRUNCATED;
        } else {
            const uint32_t v = in.peek();
            const uint32_t want = __builtin_bswap32(v);
            if (want != ((o.b << 16) | o.a)) status = PYAS_INFLATE_BAD_CHECKSUM;
        }
    }
    if (lane == 0) {
        x.status[c] = status;
        x.out_sizes[c] = o.pos;
    }
#ifdef PYAS_INFLATE_PROF
    PYAS_PROF(7);
    if (c < 4 && lane == 0)
    {
        printf("inflate stream %d out %u windows %lu: setup %lu decode %lu walk %lu scan %lu write %lu flush %lu serial %lu other %lu\n",
               (int)c, o.pos, pf_acc[8], pf_acc[0], pf_acc[1], pf_acc[2], pf_acc[3], pf_acc[4], pf_acc[5], pf_acc[6],
               pf_acc[7]);
        printf("inflate stream %d stats: symbols %lu matches %lu long %lu overlapping %lu src_in_window %lu slow %lu bytes %lu far %lu\n",
               (int)c, pf_st[0], pf_st[1], pf_st[2], pf_st[3], pf_st[4], pf_st[5], pf_st[6], pf_st[7]);
    }
#endif
}

hipError_t launch_inflate(const InflateArgs &x, int64_t n, int wbits, hipStream_t stream) {
    switch (wbits) {
    case 15: hipLaunchKernelGGL(k_inflate<15>, dim3((uint32_t)n), dim3(64), 0, stream, x); break;
    case 14: hipLaunchKernelGGL(k_inflate<14>, dim3((uint32_t)n), dim3(64), 0, stream, x); break;
    default: hipLaunchKernelGGL(k_inflate<13>, dim3((uint32_t)n), dim3(64), 0, stream, x); break;
    }
    return hipGetLastError();
}

}  // namespace pyas
