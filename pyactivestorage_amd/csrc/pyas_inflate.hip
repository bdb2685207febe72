// pyas_inflate.hip — zlib (RFC 1950) / DEFLATE (RFC 1951) decoding on gfx950.
//
// Row f3 of the hot-path table: the reference inflates every compressed chunk
// on the host, `numcodecs.Zlib.decode` -> `zlib.decompress` (built at
// activestorage/hdf2numcodec.py:34-35, applied at activestorage/storage.py:
// 119-120).  Here one workgroup of two waves inflates one chunk stream, and a
// launch covers every chunk of a query, so thousands of streams decode
// concurrently.  DEFLATE is serial within a stream, so a stream's rate is set
// by the latency of its dependent steps; the two waves split those steps and
// run them concurrently:
//
//   * the DECODER wave (wave 0) turns the bit stream into tokens -- literal,
//     match (length, distance) or stored block -- with their output offsets,
//     into an LDS token queue.  Input comes through a 128-dword LDS ring
//     refilled one 64-dword block ahead.  Compressed blocks are decoded in
//     speculative windows: lane k decodes, at each bit offset 64 j + k of the
//     window (j < NG), the whole symbol that WOULD start there (10-bit
//     literal/length and 8-bit distance root tables whose entries carry the
//     extra-bit counts and bases), and its successor offset; the real chain
//     from offset 0 is walked on the scalar unit, one v_readlane per symbol,
//     and appended to the queue (output offsets from a wave prefix sum).
//     A code past the root table, end of block, an invalid symbol, a distance
//     before the output start, output past the capacity or truncation ends
//     the chain; the serial decoder takes that symbol and reports zlib's error.
//   * the WRITER wave (wave 1) takes up to 64 queued tokens at a time (one per
//     lane, at most kBud output bytes) and writes them into the most recent
//     2^WBITS output bytes, an LDS ring flushed to HBM in coalesced 1 KiB
//     pieces with Adler-32 folded in per flush.  A token goes once every byte
//     its source needs is written: lanes write literals and short matches, the
//     whole wave copies long or overlapping matches, and a match further back
//     than the ring reads the already-flushed output from HBM (L1-bypassing
//     loads issued before the batch's LDS work).
// Error behaviour follows zlib's inflate(): bad header, preset dictionary,
// invalid block type, stored-length mismatch, over-subscribed or incomplete
// codes, invalid symbols, distance too far back, truncated input and Adler-32
// mismatch are all reported per stream (pyas_inflate_status in pyas.h).
#include "pyas_internal.hpp"

namespace pyas {
namespace {

constexpr int kLitBits = 10, kDistBits = 8;
constexpr uint32_t kFlush = 1024;   // bytes per coalesced flush (16 per lane)
#ifndef PYAS_INFLATE_Q
#define PYAS_INFLATE_Q 1024
#endif
constexpr uint32_t kQ = PYAS_INFLATE_Q;   // token queue entries (power of two)
constexpr uint32_t kStoredTok = 0xffffu;   // len field of a stored-block token (two queue slots)

__constant__ uint8_t c_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Root-table entry (32 bits): sym | code length << 9 | extra bits << 13 |
// base << 17, where extra/base are the length (literal/length table) or
// distance (distance table) fields RFC 1951 3.2.5 attaches to the symbol, so
// a whole symbol's fields come from one LDS load.  Code length 0: the code
// is longer than the root table (canonical walk).
struct Lds {
    uint32_t lit[1 << kLitBits];
    uint32_t dist[1 << kDistBits];
    uint16_t lit_cnt[16], dist_cnt[16];
    uint16_t lit_sym[288], dist_sym[32];
    uint16_t code[320];             // canonical code per symbol (build scratch)
    uint16_t offs[16], next[16];    // build scratch
    uint8_t lens[320];              // code lengths: literal/length then distance
    int32_t status;                 // build result
};

// Token queue from the decoder wave to the writer wave.  Token t sits at
// slot t % kQ: w = len << 16 | d (a match of len bytes at distance d), len
// 0: a literal (d = the byte), len kStoredTok: a stored block of d bytes
// whose input byte offset is the next slot's w.  Output offsets are not
// queued: tokens are contiguous, so the writer takes them as a prefix sum of
// the lengths from its own position -- which doubles the queue in the same
// LDS (512 -> 1024 tokens: the decoder waited 3.3M cycles per 1 MiB stream
// on a full queue of 512, profiles/r06/inflate).
struct Queue {
    uint32_t w[kQ];
    uint32_t prod;      // tokens published by the decoder
    uint32_t cons;      // tokens the writer is done with
    uint32_t done;      // 1: the decoder finished (status, adler valid)
    int32_t status;
    uint32_t adler;     // the stream's Adler-32 trailer
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t k) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)k);
}

// LDS written by other lanes of this wave is read after this point (the
// compiler may not forward a lane's own earlier store across it).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Queue counters between the two waves (LDS, workgroup scope).
__device__ __forceinline__ uint32_t load_acq(uint32_t *p) {
    return uni(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void store_rel(uint32_t *p, uint32_t v) {
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Inclusive prefix sum over the wave, all in DPP: shifts inside each 16-lane
// row, then row_bcast:15 (rows 1 and 3 add lane 15 of the row before) and
// row_bcast:31 (rows 2 and 3 add lane 31) -- no readlanes, no SGPR round trip.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Phase timing (diagnostic build, -DPYAS_INFLATE_PROF): per-wave cycle sums
// of the phases and event counts, printed for the first streams of a launch.
#ifdef PYAS_INFLATE_PROF
#define PYAS_PROF_INIT uint64_t pf_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; uint64_t pf_last = clock64(); \
                       uint64_t pf_st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PYAS_STAT(i, v) (pf_st[i] += (v))
#define PYAS_PROF(i) do { const uint64_t pf_n = clock64(); pf_acc[i] += pf_n - pf_last; pf_last = pf_n; } while (0)
#else
#define PYAS_PROF_INIT
#define PYAS_PROF(i) do { } while (0)
#define PYAS_STAT(i, v) ((void)0)
#endif

// ---------------------------------------------------------------------------
// Decoder side
// ---------------------------------------------------------------------------

// Bit reader over dword-aligned input, staged through a 256-dword LDS ring
// refilled 128 dwords (two per lane) at a time: window bits come from LDS, so
// the symbol loop waits on a global load once per refill (every ~4 KiB of
// input).  (A block loaded one refill ahead into a VGPR did not hide that
// latency: the no-refill path's copy of the loop-carried register waited on
// the load in the very next window.)
constexpr uint32_t kInRing = 256, kInBlock = 128;

struct BitIn {
    const uint32_t *w;
    uint32_t nwords;   // readable dwords from w
    uint32_t nbits;    // valid bits from w (stream end)
    uint32_t pos;      // bit position from w
    uint32_t filled;   // dwords [filled - kInRing, filled) are in the ring
    uint32_t *ring;    // LDS

    __device__ __forceinline__ uint32_t load(uint32_t k) const {
        const uint32_t i = k + (threadIdx.x & 63);
        return i < nwords ? __builtin_nontemporal_load(w + i) : 0u;
    }
    __device__ __forceinline__ void refill() {
        const uint32_t a = load(filled), b = load(filled + 64u);
        ring[(filled + (threadIdx.x & 63)) & (kInRing - 1)] = a;
        ring[(filled + 64u + (threadIdx.x & 63)) & (kInRing - 1)] = b;
        filled += kInBlock;
    }
    __device__ __forceinline__ void seek() {   // at the start and after stored blocks
        filled = pos >> 5;
        refill();
    }
    __device__ __forceinline__ void ensure() {
        if ((pos >> 5) + 64u > filled) refill();
    }
    // 32 bits at pos + off (LSB first), per lane
    __device__ __forceinline__ uint32_t bits_at(uint32_t off) const {
        const uint32_t t = pos + off, k = t >> 5;
        return __builtin_amdgcn_alignbit(ring[(k + 1) & (kInRing - 1)], ring[k & (kInRing - 1)], t & 31);
    }
    // At least 32 valid bits starting at pos (uniform).
    __device__ __forceinline__ uint32_t peek() {
        ensure();
        wave_lds_sync();
        return uni(bits_at(0));
    }
};

// Length (kind 1) or distance (kind 2) fields of symbol s for the root-table
// entry: extra bits << 13 | base << 17 (RFC 1951 3.2.5).
__device__ __forceinline__ uint32_t sym_fields(int kind, uint32_t s) {
    if (kind == 1 && s >= 257u && s < 286u) {
        const uint32_t ls = s - 257u;
        const uint32_t le = (ls < 8u || ls == 28u) ? 0u : (ls - 4u) >> 2;
        const uint32_t base = ls < 8u ? ls + 3u : ls == 28u ? 258u : ((4u + (ls & 3u)) << le) + 3u;
        return (le << 13) | (base << 17);
    }
    if (kind == 2 && s < 30u) {
        const uint32_t de = s < 4u ? 0u : (s - 2u) >> 1;
        const uint32_t base = s < 4u ? s + 1u : ((2u + (s & 1u)) << de) + 1u;
        return (de << 13) | (base << 17);
    }
    return 0u;
}

// Canonical Huffman table for `n` code lengths in L.lens[first..first+n).
// kind: 0 code-length code, 1 literal/length, 2 distance.  Returns 0, or
// PYAS_INFLATE_BAD_CODE for over-subscribed / disallowed incomplete sets
// (zlib inflate_table rules: incomplete only for a single length-1 code in
// the literal/length and distance trees).
__device__ int build(Lds &L, int first, int n, uint16_t *cnt, uint16_t *sorted, uint32_t *tab, int P, int kind) {
    const int lane = threadIdx.x & 63;
    for (int k = lane; k < (1 << P); k += 64) tab[k] = 0;
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
        if (left > 0 && max > 0 && (kind == 0 || max != 1)) status = PYAS_INFLATE_BAD_CODE;
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
        L.status = status;
    }
    wave_lds_sync();
    // end of block and the invalid symbols (literal/length 286-287, distance
    // 30-31) get no root entry: they take the canonical walk, so a root hit
    // is always an ordinary literal, length or distance
    const int n_fast = kind == 1 ? 286 : kind == 2 ? 30 : n;
    for (int s = lane; s < n; s += 64) {
        const int l = L.lens[first + s];
        if (l && l <= P && s < n_fast && !(kind == 1 && s == 256)) {
            const uint32_t rc = __builtin_bitreverse32((uint32_t)L.code[s]) >> (32 - l);
            const uint32_t e = (uint32_t)s | ((uint32_t)l << 9) | sym_fields(kind, (uint32_t)s);
            for (uint32_t k = rc; k < (1u << P); k += 1u << l) tab[k] = e;
        }
    }
    wave_lds_sync();
    return (int)uni((uint32_t)L.status);
}

// Decode one symbol: table hit, else canonical walk over the peeked bits.
// Returns sym and sets len (0 on an invalid code).
__device__ __forceinline__ uint32_t decode(uint32_t bits, const uint32_t *tab, int P, const uint16_t *cnt,
                                           const uint16_t *sorted, uint32_t &len) {
    const uint32_t e = uni(tab[bits & ((1u << P) - 1)]);
    if ((e >> 9) & 15u) {
        len = (e >> 9) & 15u;
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

template <int NG>
__device__ void decoder(const InflateArgs &x, int64_t c, Lds &L, uint32_t *in_ring, Queue &Q) {
    PYAS_PROF_INIT
    const int lane = threadIdx.x & 63;
    const uint8_t *src = x.src + x.src_offsets[c];
    const int64_t n_in = x.src_sizes[c];
    const uint32_t mis = (uint32_t)((uintptr_t)src & 3);
    BitIn in;
    in.ring = in_ring;
    in.w = reinterpret_cast<const uint32_t *>(src - mis);
    in.nbits = (uint32_t)((n_in + mis) * 8);
    in.nwords = (uint32_t)((n_in + mis + 3) / 4);
    in.pos = mis * 8;
    in.seek();
    const uint32_t cap = (uint32_t)x.dst_capacity[c];
    uint32_t q = 0;           // output bytes decoded so far
    uint32_t prod = 0;        // tokens published
    uint32_t cons_seen = 0;   // the writer's count, last read
    int status = PYAS_INFLATE_OK;
    uint32_t adler = 0;

    // wait until n more tokens fit in the queue
    auto room = [&](uint32_t n) {
        while (prod + n - cons_seen > kQ) {
            __builtin_amdgcn_s_sleep(1);
            cons_seen = load_acq(&Q.cons);
        }
    };
    auto publish = [&](uint32_t n) {
        prod += n;
        store_rel(&Q.prod, prod);
    };
    auto emit1 = [&](uint32_t w) {   // one token from the serial decoder
        room(1);
        if (lane == 0) Q.w[prod & (kQ - 1)] = w;
        publish(1);
    };

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
        if (type == 0) {   // stored: one token, the writer copies the bytes
            in.pos = (in.pos + 7) & ~7u;
            h = in.peek();
            const uint32_t len = h & 0xffffu, nlen = h >> 16;
            in.pos += 32;
            if ((len ^ 0xffffu) != nlen) { status = PYAS_INFLATE_BAD_STORED; break; }
            if (in.pos + len * 8 > in.nbits) { status = PYAS_INFLATE_TRUNCATED; break; }
            if (q + len > cap) { status = PYAS_INFLATE_OVERFLOW; break; }
            if (len) {
                room(2);
                if (lane == 0) {
                    Q.w[prod & (kQ - 1)] = (kStoredTok << 16) | len;
                    Q.w[(prod + 1) & (kQ - 1)] = in.pos >> 3;   // input byte offset from in.w
                }
                publish(2);
                q += len;
            }
            in.pos += len * 8;
            in.seek();
            continue;
        }
        if (type == 1) {   // fixed codes (RFC 1951 3.2.6)
            for (int s = lane; s < 320; s += 64)
                L.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
            wave_lds_sync();
            build(L, 0, 288, L.lit_cnt, L.lit_sym, L.lit, kLitBits, 1);
            build(L, 288, 32, L.dist_cnt, L.dist_sym, L.dist, kDistBits, 2);
        } else if (type == 2) {   // dynamic codes
            h = in.peek();
            const uint32_t nlen = (h & 31u) + 257, ndist = ((h >> 5) & 31u) + 1, ncode = ((h >> 10) & 15u) + 4;
            in.pos += 14;
            if (nlen > 286 || ndist > 30) { status = PYAS_INFLATE_BAD_CODE; break; }
            // code-length code: 3 bits per length in c_clen_order
            h = in.peek();
            in.pos += 30;
            const uint32_t h2 = in.peek();
            in.pos -= 30;
            for (int s = lane; s < 19; s += 64) {
                const uint32_t bit = 3u * (uint32_t)s;
                uint32_t v = 0;
                if ((uint32_t)s < ncode) v = bit < 30 ? (h >> bit) & 7u : (h2 >> (bit - 30)) & 7u;
                L.lens[c_clen_order[s]] = (uint8_t)v;
            }
            in.pos += 3 * ncode;
            wave_lds_sync();
            // the code-length tree uses the distance table slots (7-bit codes)
            if (build(L, 0, 19, L.dist_cnt, L.dist_sym, L.dist, 7, 0)) { status = PYAS_INFLATE_BAD_CODE; break; }
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
            wave_lds_sync();
            if (L.lens[256] == 0) { status = PYAS_INFLATE_BAD_CODE; break; }
            if (build(L, 0, 288, L.lit_cnt, L.lit_sym, L.lit, kLitBits, 1) ||
                build(L, 288, 32, L.dist_cnt, L.dist_sym, L.dist, kDistBits, 2)) {
                status = PYAS_INFLATE_BAD_CODE;
                break;
            }
        } else {
            status = PYAS_INFLATE_BAD_BLOCK;
            break;
        }
        PYAS_PROF(5);
        // One symbol, any code length (canonical walk past the root tables),
        // queued as a token.  Returns 0 = continue, 1 = end of block, 2 =
        // error (status set).
        auto one_symbol = [&]() -> int {
            if (in.pos > in.nbits) { status = PYAS_INFLATE_TRUNCATED; return 2; }
            uint32_t bits = in.peek();
            uint32_t l;
            uint32_t sym = decode(bits, L.lit, kLitBits, L.lit_cnt, L.lit_sym, l);
            if (!l) { status = PYAS_INFLATE_BAD_SYMBOL; return 2; }
            if (sym < 256) {
                if (q >= cap) { status = PYAS_INFLATE_OVERFLOW; return 2; }
                emit1(sym);
                q++;
                in.pos += l;
                return 0;
            }
            if (sym == 256) { in.pos += l; return 1; }
            if (sym >= 286) { status = PYAS_INFLATE_BAD_SYMBOL; return 2; }
            const uint32_t lf = sym_fields(1, sym);
            const uint32_t le = (lf >> 13) & 15u;
            const uint32_t len = (lf >> 17) + ((bits >> l) & ((1u << le) - 1u));
            in.pos += l + le;
            bits = in.peek();
            const uint32_t ds = decode(bits, L.dist, kDistBits, L.dist_cnt, L.dist_sym, l);
            if (!l || ds >= 30) { status = PYAS_INFLATE_BAD_SYMBOL; return 2; }
            const uint32_t df = sym_fields(2, ds);
            const uint32_t de = (df >> 13) & 15u;
            const uint32_t d = (df >> 17) + ((bits >> l) & ((1u << de) - 1u));
            in.pos += l + de;
            if (d > q) { status = PYAS_INFLATE_BAD_DISTANCE; return 2; }
            if (q + len > cap) { status = PYAS_INFLATE_OVERFLOW; return 2; }
            emit1((len << 16) | d);
            q += len;
            return 0;
        };
        // ---- speculative windows ------------------------------------------
        constexpr uint32_t kStop = 1u << 12;
        const uint32_t *lit = L.lit, *dist = L.dist;
        bool eob = false;
        uint32_t windows_left = in.nbits + 64u;   // every window consumes input; a stuck walk ends here
        while (!eob) {
            if (windows_left-- == 0u) { status = PYAS_INFLATE_BAD_SYMBOL; break; }
            in.ensure();                                 // the ring holds the window's bits
            wave_lds_sync();
            const uint32_t t0 = in.pos + (uint32_t)lane;
            const uint32_t k0 = t0 >> 5, sh = t0 & 31u;
            uint32_t dw[2 * NG + 1];
#pragma unroll
            for (int i = 0; i < 2 * NG + 1; ++i) dw[i] = in_ring[(k0 + (uint32_t)i) & (kInRing - 1)];
            uint32_t nxt[NG], olen[NG], tw[NG];
#pragma unroll
            for (int j = 0; j < NG; ++j) {
                const uint32_t lo = __builtin_amdgcn_alignbit(dw[2 * j + 1], dw[2 * j], sh);
                const uint32_t hi = __builtin_amdgcn_alignbit(dw[2 * j + 2], dw[2 * j + 1], sh);
                const uint32_t E = lit[lo & ((1u << kLitBits) - 1u)];
                const uint32_t l = (E >> 9) & 15u, sym = E & 511u, le = (E >> 13) & 15u, lbase = E >> 17;
                const uint32_t s1 = l + le;
                const uint32_t db = __builtin_amdgcn_alignbit(hi, lo, s1);   // bits after the length
                const uint32_t D = dist[db & ((1u << kDistBits) - 1u)];
                const uint32_t dl = (D >> 9) & 15u, ds = D & 511u, de = (D >> 13) & 15u, dbase = D >> 17;
                const uint32_t ml = lbase + ((lo >> l) & ((1u << le) - 1u));
                const uint32_t md = dbase + ((db >> dl) & ((1u << de) - 1u));
                const uint32_t off = 64u * (uint32_t)j + (uint32_t)lane;
                const bool is_lit = sym < 256u;
                (void)ds;
                const bool stop = in.pos + off > in.nbits || !l || (!is_lit && !dl);
                nxt[j] = stop ? kStop : is_lit ? off + l : off + s1 + dl + de;
                olen[j] = is_lit ? 1u : ml;
                tw[j] = is_lit ? sym : (ml << 16) | md;
            }
            PYAS_PROF(0);
            // the chain from offset 0, group by group (it only moves forward)
            uint64_t M[NG];
            uint32_t off = 0, prev = 0;
            bool stopped = false;
#pragma unroll
            for (int j = 0; j < NG; ++j) {
                M[j] = 0ull;
                if (!stopped) {
                    const uint32_t gb = 64u * (uint32_t)j, ge = gb + 64u;
                    while (off < ge) {
                        M[j] |= 1ull << (off - gb);
                        prev = off;
                        off = rl(nxt[j], off - gb);
                    }
                    stopped = off >= kStop;
                }
            }
            if (stopped) {                               // the stop symbol is not consumed
#pragma unroll
                for (int j = 0; j < NG; ++j)
                    if ((prev >> 6) == (uint32_t)j) M[j] &= ~(1ull << (prev & 63u));
                off = prev;
            }
            PYAS_PROF(1);
            // the window's output: past the first 32 KiB no distance reaches
            // before the output start, and a window whose whole output fits
            // the capacity has no token past it -- then one wave sum is all
            // the window needs (the writer takes offsets as its own prefix sum)
            uint32_t lsum = 0;
#pragma unroll
            for (int j = 0; j < NG; ++j) lsum += ((M[j] >> lane) & 1ull) ? olen[j] : 0u;
            uint32_t T = rl(wave_incl_sum(lsum), 63), cut = kStop;
            if (q < 32768u || q + T > cap) {
                // output offsets along the chain: two groups per 32-bit prefix sum
                uint32_t excl[NG], tot = 0;
#pragma unroll
                for (int j = 0; j < NG; j += 2) {
                    const uint32_t va = ((M[j] >> lane) & 1ull) ? olen[j] : 0u;
                    uint32_t vb = 0;
                    if (j + 1 < NG) vb = ((M[j + 1] >> lane) & 1ull) ? olen[j + 1] : 0u;
                    const uint32_t inc = wave_incl_sum(va | (vb << 16));
                    const uint32_t tt = rl(inc, 63);
                    excl[j] = tot + (inc & 0xffffu) - va;
                    tot += tt & 0xffffu;
                    if (j + 1 < NG) {
                        excl[j + 1] = tot + (inc >> 16) - vb;
                        tot += tt >> 16;
                    }
                }
                // the first chain symbol reaching before the output start or past
                // the capacity ends the chain (the serial decoder reports it)
                T = tot;
                bool bad_any = false;
#pragma unroll
                for (int j = 0; j < NG; ++j) {
                    const uint32_t a = q + excl[j];
                    bad_any = bad_any || (((M[j] >> lane) & 1ull) &&
                                          (a + olen[j] > cap || (olen[j] > 1u && (tw[j] & 0xffffu) > a)));
                }
                if (__ballot(bad_any)) {   // rare: find the first such symbol in chain order
#pragma unroll
                    for (int j = 0; j < NG; ++j) {
                        const bool on = (M[j] >> lane) & 1ull;
                        const uint32_t a = q + excl[j];
                        const uint64_t b = __ballot(on && (a + olen[j] > cap || (olen[j] > 1u && (tw[j] & 0xffffu) > a)));
                        if (b && cut == kStop) {
                            const uint32_t cc = (uint32_t)__builtin_ctzll(b);
                            cut = 64u * (uint32_t)j + cc;
                            T = rl(excl[j], cc);
                        }
                    }
                }
            }
            if (cut != kStop) {
#pragma unroll
                for (int j = 0; j < NG; ++j) {
                    const uint32_t lo = 64u * (uint32_t)j;
                    M[j] = cut <= lo ? 0ull : cut - lo >= 64u ? M[j] : M[j] & ((1ull << (cut - lo)) - 1ull);
                }
                off = cut;
            }
            uint32_t count = 0;
#pragma unroll
            for (int j = 0; j < NG; ++j) count += (uint32_t)__builtin_popcountll(M[j]);
            PYAS_PROF(2);
            room(count);
            PYAS_PROF(3);
            uint32_t base = prod;
#pragma unroll
            for (int j = 0; j < NG; ++j) {
                if ((M[j] >> lane) & 1ull) {
                    const uint32_t idx = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(M[j] >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)M[j], 0u));
                    Q.w[idx & (kQ - 1)] = tw[j];
                }
                base += (uint32_t)__builtin_popcountll(M[j]);
            }
            publish(count);
            PYAS_STAT(0, 1u);
            PYAS_STAT(1, count);
            q += T;
            in.pos += off;
            PYAS_PROF(2);
            if (stopped || cut != kStop) {
                PYAS_STAT(2, 1u);
                const int r = one_symbol();
                PYAS_PROF(4);
                if (r == 2) break;
                if (r == 1) eob = true;
            }
        }
    }
    if (status == 0) {   // the Adler-32 trailer
        in.pos = (in.pos + 7) & ~7u;
        if (in.pos + 32 > in.nbits) status = PYAS_INFLATE_TRUNCATED;
        else adler = __builtin_bswap32(in.peek());
    }
    if (lane == 0) {
        Q.status = status;
        Q.adler = adler;
    }
    store_rel(&Q.done, 1u);
#ifdef PYAS_INFLATE_PROF
    PYAS_PROF(7);
    if (c < 4 && lane == 0)
        printf("decoder %d: decode %lu walk %lu scan+emit %lu queue-full %lu serial %lu blocks %lu end %lu | windows %lu "
               "tokens %lu serial %lu\n",
               (int)c, pf_acc[0], pf_acc[1], pf_acc[2], pf_acc[3], pf_acc[4], pf_acc[5], pf_acc[7], pf_st[0], pf_st[1],
               pf_st[2]);
#endif
}

// ---------------------------------------------------------------------------
// Writer side
// ---------------------------------------------------------------------------

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
        // s = sum b_k, t = sum (n - 16 lane - k) b_k: byte dot products
        s = __builtin_amdgcn_udot4(v.x, 0x01010101u, 0u, false) + __builtin_amdgcn_udot4(v.y, 0x01010101u, 0u, false) +
            __builtin_amdgcn_udot4(v.z, 0x01010101u, 0u, false) + __builtin_amdgcn_udot4(v.w, 0x01010101u, 0u, false);
        uint32_t kb = __builtin_amdgcn_udot4(v.x, 0x03020100u, 0u, false);
        kb = __builtin_amdgcn_udot4(v.y, 0x07060504u, kb, false);
        kb = __builtin_amdgcn_udot4(v.z, 0x0b0a0908u, kb, false);
        kb = __builtin_amdgcn_udot4(v.w, 0x0f0e0d0cu, kb, false);
        t = (n - (uint32_t)lane * 16u) * s - kb;
    } else {
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t byte = win[(o.fpos + i) & MASK];
            o.dst[o.fpos + i] = (uint8_t)byte;
            s += byte;
            t += (n - i) * byte;
        }
    }
    // wave sums in DPP (shfl_xor steps are LDS round trips: ~1k cycles a
    // flush); n <= 1024 keeps every sum below 2^32 (t <= 1024^2 * 255 / 2)
    s = rl(wave_incl_sum(s), 63);
    t = rl(wave_incl_sum(t), 63);
    // a' = a + sum b_i;  b' = b + n*a + sum (n - i) b_i   (mod 65521)
    const uint32_t bb = o.b + n * o.a + t;
    o.a = (o.a + s) % 65521u;
    o.b = bb % 65521u;
    o.fpos += n;
}

// 16 bytes of already-flushed output at dst + src (realigned from five
// L1-bypassing dword loads; dwords at or past `lim` are not read).
struct Far16 {
    uint32_t v[5], sh;
    __device__ __forceinline__ void load(const uint8_t *p, const uint8_t *lim) {
        const uint32_t *wb = reinterpret_cast<const uint32_t *>((uintptr_t)p & ~(uintptr_t)3);
        sh = (uint32_t)((uintptr_t)p & 3);
#pragma unroll
        for (int k = 0; k < 5; ++k)
            v[k] = reinterpret_cast<const uint8_t *>(wb + k) < lim
                       ? __hip_atomic_load(wb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0u;
    }
    __device__ __forceinline__ uint32_t word(int k) const { return __builtin_amdgcn_alignbyte(v[k + 1], v[k], sh); }
};

template <int WBITS>
__device__ void writer(const InflateArgs &x, int64_t c, uint8_t *win, Queue &Q) {
    PYAS_PROF_INIT
    constexpr uint32_t kWin = 1u << WBITS, kWinMask = kWin - 1;
    // A batch writes at most kBud bytes past o.pos and starts with fewer than
    // kFlush bytes unflushed, so a source d <= kFar back is still in the ring
    // and a longer one is already in dst; the ring holds the unflushed bytes.
    constexpr uint32_t kBud = kWin / 8, kFar = kWin - kBud;
    static_assert(kFar > 258u + kBud + kFlush, "far sources must be flushed");
    const int lane = threadIdx.x & 63;
    uint32_t *win32 = reinterpret_cast<uint32_t *>(win);
    const uint8_t *src = x.src + x.src_offsets[c];
    const uint32_t mis = (uint32_t)((uintptr_t)src & 3);
    const uint32_t *inw = reinterpret_cast<const uint32_t *>(src - mis);
    const uint32_t in_words = (uint32_t)((x.src_sizes[c] + mis + 3) / 4);
    Out o;
    o.dst = x.dst + x.dst_offsets[c];
    o.cap = (uint32_t)x.dst_capacity[c];
    o.pos = o.fpos = 0;
    o.a = 1;
    o.b = 0;
    o.aligned = (((uintptr_t)o.dst) & 15) == 0;
    int status = PYAS_INFLATE_OK;
    uint32_t cons = 0;

    // Whole-wave copy of one match (tp, td, tl): every source byte lies before
    // tp (td >= tl) or repeats the period [tp - td, tp) (td < tl).
    // (All reads are issued unconditionally -- ring indices are masked -- so
    // they are in flight together; the writes are predicated.)
    auto wave_copy = [&](uint32_t tp, uint32_t td, uint32_t tl) {
        const uint32_t ts = tp - td;
        uint32_t m = (uint32_t)lane, r64 = 64u;
        if (td < tl) {
            r64 = 64u % td;
            m = (uint32_t)lane % td;
        }
        if (tl <= 64u) {
            const uint32_t v = win[(ts + m) & kWinMask];
            if ((uint32_t)lane < tl) win[(tp + (uint32_t)lane) & kWinMask] = (uint8_t)v;
            return;
        }
        uint32_t idx[5];
#pragma unroll
        for (uint32_t k = 0; k < 5u; ++k) {
            idx[k] = ts + m;
            m += r64;
            m = (td < tl && m >= td) ? m - td : m;
        }
        uint32_t v[5];
#pragma unroll
        for (uint32_t k = 0; k < 5u; ++k) v[k] = win[idx[k] & kWinMask];
#pragma unroll
        for (uint32_t k = 0; k < 5u; ++k) {
            const uint32_t ii = (uint32_t)lane + 64u * k;
            if (ii < tl) win[(tp + ii) & kWinMask] = (uint8_t)v[k];
        }
    };

    for (;;) {
        uint32_t prod = 0, done = 0;
        for (;;) {
            done = load_acq(&Q.done);
            prod = load_acq(&Q.prod);
            if (prod - cons >= 64u || done) break;
            __builtin_amdgcn_s_sleep(2);
        }
        PYAS_PROF(0);
        if (done && Q.status != PYAS_INFLATE_OK) {
            status = Q.status;
            break;
        }
        if (prod == cons) break;   // done, every token written
#ifdef PYAS_INFLATE_DECODE_ONLY
        cons = prod;               // diagnostic: the decoder alone
        store_rel(&Q.cons, cons);
        continue;
#endif
        const uint32_t avail = prod - cons;
        const bool act = (uint32_t)lane < avail;
        const uint32_t slot = (cons + (uint32_t)lane) & (kQ - 1);
        const uint32_t w = act ? Q.w[slot] : 0u;
        uint32_t len = w >> 16, d = w & 0xffffu;
        // output offsets: the lengths' prefix sum from o.pos (lanes past a
        // stored token sum garbage; the batch ends before them)
        const uint32_t olen = act ? (len ? len : 1u) : 0u;
        const uint32_t p = o.pos + wave_incl_sum(olen) - olen;
        const uint64_t stored = __ballot(act && len == kStoredTok);
        if (stored & 1ull) {   // a stored block: 16 bytes per lane per 1 KiB step
            const uint32_t slen = rl(d, 0);
            const uint32_t byte0 = Q.w[(cons + 1) & (kQ - 1)];
            const uint32_t mine = (uint32_t)lane * 16u;
            uint32_t dn = 0;
            // head: single bytes up to a dword boundary of the output
            const uint32_t head = min((4u - (o.pos & 3u)) & 3u, slen);
            if (head) {
                while (o.pos - o.fpos >= kFlush) flush<kWinMask>(win, o, kFlush);
                if ((uint32_t)lane < head) {
                    const uint32_t b = byte0 + (uint32_t)lane;
                    const uint32_t v = __builtin_nontemporal_load(inw + (b >> 2));
                    win[(o.pos + (uint32_t)lane) & kWinMask] = (uint8_t)(v >> (8 * (b & 3u)));
                }
                o.pos += head;
                dn = head;
                wave_lds_sync();
            }
            // then 16 bytes per lane per 1 KiB step as four dword writes (the
            // output is dword-aligned; a last partial dword writes ring bytes
            // past o.pos that nothing reads before the next tokens write them),
            // kStoredSteps steps' input loads in flight at once
            constexpr uint32_t kStoredSteps = 4;
            while (dn < slen) {
                const uint32_t span = min(slen - dn, kStoredSteps * kFlush);
                uint32_t dw[kStoredSteps][5];
#pragma unroll
                for (uint32_t s = 0; s < kStoredSteps; ++s) {
                    const uint32_t b = byte0 + dn + s * kFlush + mine;
                    const uint32_t wi = b >> 2;
                    const bool on = s * kFlush + mine < span;
#pragma unroll
                    for (uint32_t k = 0; k < 5; ++k)
                        dw[s][k] = on && wi + k < in_words ? __builtin_nontemporal_load(inw + wi + k) : 0u;
                }
                const uint32_t sh = (byte0 + dn) & 3u;   // the same for every lane and step
#pragma unroll
                for (uint32_t s = 0; s < kStoredSteps; ++s) {
                    if (s * kFlush >= span) break;
                    while (o.pos - o.fpos >= kFlush) flush<kWinMask>(win, o, kFlush);
                    const uint32_t step = min(span - s * kFlush, kFlush);
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k)
                        if (mine + 4u * k < step)
                            win32[(((o.pos + mine) >> 2) + k) & (kWin / 4 - 1)] =
                                __builtin_amdgcn_alignbyte(dw[s][k + 1], dw[s][k], sh);
                    o.pos += step;
                    wave_lds_sync();
                }
                dn += span;
            }
            cons += 2;
            store_rel(&Q.cons, cons);
            PYAS_PROF(3);
            continue;
        }
        // this batch: the tokens before the first stored one, at most kBud
        // output bytes (tokens are contiguous from o.pos)
        uint32_t n = min(avail, 64u);
        if (stored) n = min(n, (uint32_t)__builtin_ctzll(stored));
        const uint64_t over = __ballot(act && p + olen - o.pos > kBud);
        if (over) n = min(n, (uint32_t)__builtin_ctzll(over));
        const bool mine = (uint32_t)lane < n;
        if (!mine) len = d = 0u;
        const uint32_t src_b = p - d;
        const bool far = mine && len && d > kFar;
        const uint32_t need = mine && len ? min(src_b + len, p) : 0u;   // [src, need) must be written
        bool done_t = !mine;
        // far sources: issue their first 16 bytes now (flushed; ready at once)
        Far16 fv;
        const bool any_far = __ballot(far) != 0ull;
        if (any_far) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's flush stores have landed
            if (far) fv.load(o.dst + src_b, o.dst + o.fpos);
        }
        PYAS_STAT(0, 1u);
        PYAS_STAT(1, n);
        PYAS_PROF(1);
        for (;;) {
            const uint64_t und = __ballot(!done_t);
            if (!und) break;
            PYAS_STAT(2, 1u);
            const uint32_t W = rl(p, (uint32_t)__builtin_ctzll(und));
            const bool ready = !done_t && need <= W;
            if (ready && !len) win[p & kWinMask] = (uint8_t)d;
            // short non-overlapping matches, one lane each: 16 source bytes
            // from five ring dwords
            const uint32_t ns = (ready && len && !far && len <= 16u && d >= len) ? len : 0u;
            if (__ballot(ns != 0u)) {
                const uint32_t wi = src_b >> 2, sh = src_b & 3u;
                uint32_t r[5];
#pragma unroll
                for (uint32_t k = 0; k < 5; ++k) r[k] = win32[(wi + k) & (kWin / 4 - 1)];
#pragma unroll
                for (uint32_t k = 0; k < 16u; ++k) {
                    if (!__ballot(k < ns)) break;
                    const uint32_t qv = __builtin_amdgcn_alignbyte(r[(k >> 2) + 1], r[k >> 2], sh);
                    if (k < ns) win[(p + k) & kWinMask] = (uint8_t)(qv >> (8 * (k & 3u)));
                }
            }
            PYAS_PROF(4);
            // far matches (ready in the first round): the prefetched 16 bytes,
            // then 16-byte steps for longer ones
            if (any_far && __ballot(ready && far)) {
                PYAS_STAT(3, __builtin_popcountll(__ballot(ready && far)));
                const uint32_t nf = (ready && far) ? len : 0u;
#pragma unroll
                for (uint32_t k = 0; k < 16u; ++k)
                    if (k < nf) win[(p + k) & kWinMask] = (uint8_t)(fv.word((int)(k >> 2)) >> (8 * (k & 3u)));
                for (uint32_t fo = 16; __ballot(fo < nf); fo += 16u) {
                    if (fo < nf) {
                        Far16 g;
                        g.load(o.dst + src_b + fo, o.dst + o.fpos);
                        const uint32_t m = min(nf - fo, 16u);
#pragma unroll
                        for (uint32_t k = 0; k < 16u; ++k)
                            if (k < m) win[(p + fo + k) & kWinMask] = (uint8_t)(g.word((int)(k >> 2)) >> (8 * (k & 3u)));
                    }
                }
            }
            PYAS_PROF(5);
            // long or overlapping matches: the whole wave, one at a time
            uint64_t coop = __ballot(ready && len && !far && (len > 16u || d < len));
            PYAS_STAT(4, __builtin_popcountll(coop));
            while (coop) {
                const uint32_t t = (uint32_t)__builtin_ctzll(coop);
                coop &= coop - 1ull;
                wave_copy(rl(p, t), rl(d, t), rl(len, t));
            }
            done_t = done_t || ready;
            wave_lds_sync();
            // the first token not written is ready now; tokens that read the
            // one before them (runs of long/overlapping matches, and short
            // ones) are taken in order by the whole wave -- any number of long
            // or overlapping ones, up to kHead others -- before the next
            // parallel round
            constexpr uint32_t kHead = 4;
            for (uint32_t h = 0;;) {
                const uint64_t u2 = __ballot(!done_t);
                if (!u2) break;
                const uint32_t t = (uint32_t)__builtin_ctzll(u2);
                const uint32_t tl = rl(len, t), td = rl(d, t);
                const bool longish = tl > 16u || (tl && td < tl);
                if (td > kFar || (!longish && h == kHead)) break;
                h += longish ? 0u : 1u;
                PYAS_STAT(5, 1u);
                const uint32_t tp = rl(p, t);
                if (tl) wave_copy(tp, td, tl);
                else if ((uint32_t)lane == t) win[tp & kWinMask] = (uint8_t)td;
                done_t = done_t || (uint32_t)lane == t;
                wave_lds_sync();
            }
            PYAS_PROF(6);
        }
        cons += n;
        store_rel(&Q.cons, cons);
        o.pos = rl(p, n - 1) + rl(olen, n - 1);
        PYAS_PROF(1);
        while (o.pos - o.fpos >= kFlush) flush<kWinMask>(win, o, kFlush);
        PYAS_PROF(2);
    }
    if (status == 0) {
        if (o.pos > o.fpos) {
            wave_lds_sync();
            while (o.pos - o.fpos >= kFlush) flush<kWinMask>(win, o, kFlush);
            if (o.pos > o.fpos) flush<kWinMask>(win, o, o.pos - o.fpos);
        }
        if (Q.adler != ((o.b << 16) | o.a)) status = PYAS_INFLATE_BAD_CHECKSUM;
    }
    if (lane == 0) {
        x.status[c] = status;
        x.out_sizes[c] = o.pos;
    }
#ifdef PYAS_INFLATE_PROF
    PYAS_PROF(7);
    if (c < 4 && lane == 0)
        printf("writer  %d out %u: wait %lu setup %lu lit+short %lu far %lu coop+chain %lu flush %lu stored %lu end %lu | "
               "batches %lu tokens %lu rounds %lu far %lu coop %lu chain %lu\n",
               (int)c, o.pos, pf_acc[0], pf_acc[1], pf_acc[4], pf_acc[5], pf_acc[6], pf_acc[2], pf_acc[3], pf_acc[7],
               pf_st[0], pf_st[1], pf_st[2], pf_st[3], pf_st[4], pf_st[5]);
#endif
}

}  // namespace

// One stream per workgroup: wave 0 decodes, wave 1 writes.  NG bit-offset
// groups per decoder window; 2^WBITS bytes of output ring.
template <int WBITS, int NG>
__global__ __launch_bounds__(128) void k_inflate(InflateArgs x) {
    __shared__ Lds L;
    __shared__ alignas(16) uint8_t win[1u << WBITS];
    __shared__ uint32_t in_ring[kInRing];
    __shared__ Queue Q;
    const int64_t c = blockIdx.x;
    if (threadIdx.x == 0) {
        Q.prod = Q.cons = Q.done = 0u;
        Q.status = 0;
        Q.adler = 0u;
    }
    __syncthreads();
    if (threadIdx.x < 64) decoder<NG>(x, c, L, in_ring, Q);
    else writer<WBITS>(x, c, win, Q);
}

// PYAS_INFLATE_NG: bit-offset groups per decoder window (1, 2 or 4; 8 took
// 150 VGPRs for the same 147 MB/s per stream, profiles/r06/inflate).  Read
// once per process.
static int inflate_ng() {
    static const int ng = [] {
        const char *v = getenv("PYAS_INFLATE_NG");
        const int g = v ? atoi(v) : 4;
        return (g == 1 || g == 2 || g == 4) ? g : 4;
    }();
    return ng;
}

template <int WBITS>
static void launch_ng(const InflateArgs &x, int64_t n, hipStream_t stream) {
    switch (inflate_ng()) {
    case 1: hipLaunchKernelGGL((k_inflate<WBITS, 1>), dim3((uint32_t)n), dim3(128), 0, stream, x); break;
    case 2: hipLaunchKernelGGL((k_inflate<WBITS, 2>), dim3((uint32_t)n), dim3(128), 0, stream, x); break;
    default: hipLaunchKernelGGL((k_inflate<WBITS, 4>), dim3((uint32_t)n), dim3(128), 0, stream, x); break;
    }
}

hipError_t launch_inflate(const InflateArgs &x, int64_t n, int wbits, hipStream_t stream) {
    switch (wbits) {
    case 15: launch_ng<15>(x, n, stream); break;
    case 14: launch_ng<14>(x, n, stream); break;
    default: launch_ng<13>(x, n, stream); break;
    }
    return hipGetLastError();
}

}  // namespace pyas
