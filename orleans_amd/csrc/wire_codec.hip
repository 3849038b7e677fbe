// wire_codec.hip — f2: received message frames -> the orl_msg_hdr records the route kernels read (gfx950).
//
// Reference (paths relative to randa1/orleans):
//   framing    Message.Serialize_Impl (src/Orleans/Messaging/Message.cs:915-951): int32 header length, int32 body
//              length, header bytes, body bytes; IncomingMessageBuffer.TryDecodeMessage (IncomingMessageBuffer.cs:
//              94-135) walks the frames — the host hands us the frame offsets it found.
//   headers    SerializationManager.DeserializeMessageHeaders (SerializationManager.cs:1773-1853) over
//              BinaryTokenStreamReader.TryReadSimpleType (BinaryTokenStreamReader.cs:489-582).
//   getters    Message.Category / TargetSilo / SendingSilo / TargetGrain / TargetActivation / TargetAddress
//              (Message.cs:149, 199-231, 251-255; GetScalarHeader / GetSimpleHeader :650-666).
// The oracle is oracle/wire_codec.py (decode_frames); statuses and their precedence are defined there.
//
// One lane per frame: each lane walks its own header sequentially.  Bytes come from 4-byte aligned words joined
// with v_alignbyte (no byte-granular loads, no read beyond the aligned word that holds a frame's last byte).
// Large batches stage every frame's header window in LDS first (k_decode_frames_pipe).  Byte/integer work only.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include "orl_internal.h"

namespace orl {

namespace {

// SerializationTokenType (SerializationTokenType.cs:30-109)
enum : uint32_t {
    T_NULL = 0, T_TRUE = 3, T_FALSE = 4, T_INT = 11, T_SHORT = 12, T_LONG = 13, T_SBYTE = 14, T_UINT = 15,
    T_USHORT = 16, T_ULONG = 17, T_BYTE = 18, T_FLOAT = 19, T_DOUBLE = 20, T_DECIMAL = 21, T_STRING = 22,
    T_CHAR = 23, T_GUID = 24, T_DATE = 25, T_TIMESPAN = 26, T_IPADDR = 27, T_IPEP = 28, T_OBJECT = 29,
    T_GRAIN = 40, T_ACT = 41, T_SILO = 42, T_ACTADDR = 43, T_CORR = 44, T_DICT = 50, T_LIST = 51,
    T_SPECIFIED = 97,
};
// Message.Header values the routing path reads (Message.cs:29-70)
enum : uint32_t { H_CATEGORY = 3, H_SENDING_SILO = 20, H_TARGET_ACTIVATION = 22, H_TARGET_GRAIN = 23, H_TARGET_SILO = 24 };

constexpr uint64_t kMaxTicks = 3155378975999999999ull;  // DateTime.MaxValue.Ticks

// Byte sources.  GlobalSrc: positions are absolute 64-bit buffer offsets; word reads are clamped to `last`, the
// word holding the current frame's last byte, so any read is inside the frame's words.  LdsSrc: one frame staged in
// an LDS row, positions are 32-bit offsets from the row start (the frame's first aligned word); a row has a spare
// word after its 64, so the second word of a read is always readable.  Both read 4 bytes with two word loads and
// v_alignbyte and no branch: ({hi, lo} >> 8 * (p & 3))[31:0].
struct GlobalSrc {
    using P = uint64_t;
    const uint32_t* __restrict__ w;
    uint64_t last;
    __device__ __forceinline__ uint32_t word(uint64_t i) const { return w[i < last ? i : last]; }
    __device__ __forceinline__ uint32_t ld32(uint64_t p) const {
        const uint64_t wi = p >> 2;
        return __builtin_amdgcn_alignbyte(word(wi + 1), word(wi), (uint32_t)(p & 3u));
    }
};
struct LdsSrc {
    using P = uint32_t;
    const uint32_t* row;
    __device__ __forceinline__ uint32_t word(uint32_t i) const { return row[i]; }
    __device__ __forceinline__ uint32_t ld32(uint32_t p) const {
        const uint32_t wi = p >> 2;
        return __builtin_amdgcn_alignbyte(row[wi + 1], row[wi], p & 3u);
    }
};

template <class S>
__device__ __forceinline__ uint32_t ld32(const S& w, typename S::P p) { return w.ld32(p); }
template <class S>
__device__ __forceinline__ uint32_t ld8(const S& w, typename S::P p) {
    return (w.word(p >> 2) >> ((uint32_t)(p & 3u) * 8u)) & 0xFFu;
}
template <class S>
__device__ __forceinline__ uint64_t ld64(const S& w, typename S::P p) {
    return (uint64_t)ld32(w, p) | ((uint64_t)ld32(w, p + 4) << 32);
}

// string.IsNullOrWhiteSpace over the UTF-8 bytes [p, p+len): whitespace-only iff the bytes split into encodings
// of Char.IsWhiteSpace code points (U+0009-000D, 0020, 0085, 00A0, 1680, 2000-200A, 2028, 2029, 202F, 205F,
// 3000).  Any other byte decodes to a non-space char or to U+FFFD.
template <class S>
__device__ bool all_whitespace(const S& w, typename S::P p, typename S::P len) {
    const typename S::P e = p + len;
    while (p < e) {
        const uint32_t b0 = ld8(w, p);
        if (b0 == 0x20u || (b0 >= 0x09u && b0 <= 0x0Du)) { p += 1; continue; }
        if (b0 == 0xC2u && p + 2 <= e) {
            const uint32_t b1 = ld8(w, p + 1);
            if (b1 == 0x85u || b1 == 0xA0u) { p += 2; continue; }
            return false;
        }
        if ((b0 == 0xE1u || b0 == 0xE2u || b0 == 0xE3u) && p + 3 <= e) {
            const uint32_t b1 = ld8(w, p + 1), b2 = ld8(w, p + 2);
            const uint32_t cp = ((b0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
            const bool cont = (b1 & 0xC0u) == 0x80u && (b2 & 0xC0u) == 0x80u;
            const bool ws = cp == 0x1680u || (cp >= 0x2000u && cp <= 0x200Au) || cp == 0x2028u || cp == 0x2029u ||
                            cp == 0x202Fu || cp == 0x205Fu || cp == 0x3000u;
            if (cont && ws) { p += 3; continue; }
            return false;
        }
        return false;
    }
    return true;
}

// Strict UTF-8 (RFC 3629: no overlongs, no surrogates, <= U+10FFFF) — the byte strings .NET's decoder maps to
// themselves when re-encoded.
template <class S>
__device__ bool strict_utf8(const S& w, typename S::P p, typename S::P len) {
    const typename S::P e = p + len;
    while (p < e) {
        if (p + 4 <= e && (ld32(w, p) & 0x80808080u) == 0) { p += 4; continue; }  // four ASCII bytes
        const uint32_t b0 = ld8(w, p);
        if (b0 < 0x80u) { p += 1; continue; }
        uint32_t n, lo = 0x80u, hi = 0xBFu;
        if (b0 >= 0xC2u && b0 <= 0xDFu) n = 1;
        else if (b0 >= 0xE0u && b0 <= 0xEFu) { n = 2; if (b0 == 0xE0u) lo = 0xA0u; if (b0 == 0xEDu) hi = 0x9Fu; }
        else if (b0 >= 0xF0u && b0 <= 0xF4u) { n = 3; if (b0 == 0xF0u) lo = 0x90u; if (b0 == 0xF4u) hi = 0x8Fu; }
        else return false;
        if (p + 1 + n > e) return false;
        const uint32_t b1 = ld8(w, p + 1);
        if (b1 < lo || b1 > hi) return false;
        for (uint32_t j = 2; j <= n; ++j)
            if ((ld8(w, p + j) & 0xC0u) != 0x80u) return false;
        p += 1 + n;
    }
    return true;
}

// JenkinsHash.ComputeHash(byte[]) (JenkinsHash.cs:68-115) over [p, p+len).
template <class S>
__device__ uint32_t jenkins_stream(const S& w, typename S::P p, uint32_t len) {
    uint32_t a = 0x9e3779b9u, b = 0x9e3779b9u, c = 0u;
    uint32_t i = 0;
    for (; i + 12u <= len; i += 12u) {
        a += ld32(w, p + i);
        b += ld32(w, p + i + 4);
        c += ld32(w, p + i + 8);
        ORL_MIX(a, b, c);
    }
    c += len;
    const uint32_t t = len - i;  // 0..11 tail bytes: 0-3 -> a, 4-7 -> b, 8-10 -> c << 8
    auto mask = [](uint32_t k) { return k >= 4 ? 0xFFFFFFFFu : (1u << (8u * k)) - 1u; };
    a += ld32(w, p + i) & mask(t);
    b += ld32(w, p + i + 4) & mask(t > 4 ? t - 4 : 0);
    c += (ld32(w, p + i + 8) & mask(t > 8 ? t - 8 : 0)) << 8;
    ORL_MIX(a, b, c);
    return c;
}

// ReadUniqueKey (:424-431) + UniqueKey.ValidateKeyExt (UniqueKey.cs:328-350).  Advances p; returns a status.
template <bool CANON = false, class S>
__device__ __forceinline__ uint32_t skip_unique_key(const S& w, typename S::P end, typename S::P& p, bool* noncanon = nullptr) {
    if (p + 28 > end) return ORL_DEC_MALFORMED;
    const uint32_t cat = ld32(w, p + 20) >> 24;  // top byte of TypeCodeData
    const int32_t len = (int32_t)ld32(w, p + 24);
    p += 28;
    if (len == -1) return cat == 6u ? ORL_DEC_MALFORMED : ORL_DEC_OK;  // KeyExt grain needs an extension
    if (len < 0 || p + (typename S::P)len > end) return ORL_DEC_MALFORMED;
    if (cat != 6u) return ORL_DEC_MALFORMED;                             // extension on a non-KeyExt key
    if (all_whitespace(w, p, (typename S::P)len)) return ORL_DEC_MALFORMED;
    if (CANON && !strict_utf8(w, p, (typename S::P)len)) *noncanon = true;
    p += (typename S::P)len;
    return ORL_DEC_OK;
}

template <class S>
__device__ __forceinline__ bool port_ok(const S& w, typename S::P p) {
    return ld32(w, p) <= 65535u;  // new IPEndPoint(addr, port): 0 <= port <= 65535
}

// One header value (DeserializeMessageHeaderHelper :1833-1853), starting at its token.  Lists are flattened
// with a pending-value counter (a list only adds values), so nesting depth costs no state.
// CANON (the stamp path): also flag, in *noncanon, a string or KeyExt that is not strict UTF-8 — re-serializing it
// would not give its bytes back.
template <bool CANON = false, class S>
__device__ uint32_t skip_value(const S& w, typename S::P end, typename S::P& p, bool* noncanon = nullptr) {
    uint64_t pending = 1;
    while (pending) {
        --pending;
        if (p >= end) return ORL_DEC_MALFORMED;
        const uint32_t t = ld8(w, p);
        p += 1;
        typename S::P sz = 0;
        switch (t) {
        case T_NULL: case T_TRUE: case T_FALSE: case T_OBJECT: sz = 0; break;
        case T_SBYTE: case T_BYTE: sz = 1; break;
        case T_SHORT: case T_USHORT: sz = 2; break;
        case T_INT: case T_UINT: case T_FLOAT: sz = 4; break;
        case T_LONG: case T_ULONG: case T_DOUBLE: case T_TIMESPAN: case T_CORR: sz = 8; break;
        case T_GUID: case T_IPADDR: sz = 16; break;
        case T_CHAR:  // Convert.ToChar(short) throws for a negative short
            if (p + 2 > end) return ORL_DEC_MALFORMED;
            if (ld8(w, p + 1) & 0x80u) return ORL_DEC_MALFORMED;
            sz = 2;
            break;
        case T_DECIMAL: {  // new decimal(int[]): flags = sign | scale<<16, scale <= 28
            if (p + 16 > end) return ORL_DEC_MALFORMED;
            const uint32_t f = ld32(w, p + 12);
            if ((f & 0x7F00FFFFu) || ((f >> 16) & 0xFFu) > 28u) return ORL_DEC_MALFORMED;
            sz = 16;
            break;
        }
        case T_DATE: {  // DateTime.FromBinary: local kinds depend on the host time zone
            if (p + 8 > end) return ORL_DEC_MALFORMED;
            const uint64_t v = ld64(w, p);
            if (v >> 63) return ORL_DEC_UNSUPPORTED;
            if ((v & 0x3FFFFFFFFFFFFFFFull) > kMaxTicks) return ORL_DEC_MALFORMED;
            sz = 8;
            break;
        }
        case T_IPEP:
            if (p + 20 > end || !port_ok(w, p + 16)) return ORL_DEC_MALFORMED;
            sz = 20;
            break;
        case T_SILO:
            if (p + 24 > end || !port_ok(w, p + 16)) return ORL_DEC_MALFORMED;
            sz = 24;
            break;
        case T_STRING: {
            if (p + 4 > end) return ORL_DEC_MALFORMED;
            const int32_t len = (int32_t)ld32(w, p);
            if (len < -1) return ORL_DEC_MALFORMED;
            sz = 4 + (len > 0 ? (typename S::P)len : 0);
            if (CANON && len > 0 && p + sz <= end && !strict_utf8(w, p + 4, (typename S::P)len)) *noncanon = true;
            break;
        }
        case T_GRAIN: case T_ACT: {
            const uint32_t st = skip_unique_key<CANON>(w, end, p, noncanon);
            if (st) return st;
            continue;
        }
        case T_ACTADDR: {
            if (p + 24 > end || !port_ok(w, p + 16)) return ORL_DEC_MALFORMED;
            p += 24;
            uint32_t st = skip_unique_key<CANON>(w, end, p, noncanon);
            if (!st) st = skip_unique_key<CANON>(w, end, p, noncanon);
            if (st) return st;
            continue;
        }
        case T_LIST: {
            if (p + 4 > end) return ORL_DEC_MALFORMED;
            const int32_t cnt = (int32_t)ld32(w, p);
            if (cnt < 0) return ORL_DEC_MALFORMED;
            pending += (uint64_t)cnt;
            sz = 4;
            break;
        }
        case T_DICT: return ORL_DEC_UNSUPPORTED;       // nested header dictionary: host path
        case T_SPECIFIED: return ORL_DEC_UNSUPPORTED;  // registered serializer: host path
        default: return ORL_DEC_MALFORMED;             // "Unexpected token ... parsing message headers"
        }
        if (p + sz > end) return ORL_DEC_MALFORMED;
        p += sz;
    }
    return ORL_DEC_OK;
}

template <class S>
__device__ uint32_t silo_lookup(const SiloAddrEntry* __restrict__ tab, const S& w, typename S::P p) {
    uint32_t a[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) a[i] = ld32(w, p + 4u * i);
    uint32_t s = silo_addr_slot(a);
    for (uint32_t probe = 0; probe < kSiloAddrSlots; ++probe) {
        const SiloAddrEntry& e = tab[s];
        if (e.silo == 0xFFu) return 0xFFu;
        if (e.w[0] == a[0] && e.w[1] == a[1] && e.w[2] == a[2] && e.w[3] == a[3] && e.w[4] == a[4] && e.w[5] == a[5])
            return e.silo;
        s = (s + 1u) & (kSiloAddrSlots - 1u);
    }
    return 0xFFu;
}

// Token classes for the common-case entry loop: the fixed byte count after the token plus what else the reader
// checks.  Rare or nested tokens (CLS_SLOW) go through skip_value, which restates every reader rule.
enum : uint32_t {
    CLS_SIZE = 63u,
    CLS_STR = 1u << 6,    // + max(int32 length at +0, 0); length < -1 throws
    CLS_KEY = 1u << 7,    // UniqueKey: + max(int32 length at +24, 0); ValidateKeyExt on the category byte at +23
    CLS_PORT = 1u << 8,   // int32 port at +16 must be in [0, 65535]
    CLS_DATE = 1u << 9,   // DateTime.FromBinary rules
    CLS_SLOW = 1u << 10,
};
__device__ uint32_t token_class(uint32_t t) {
    switch (t) {
    case T_NULL: case T_TRUE: case T_FALSE: case T_OBJECT: return 0;
    case T_SBYTE: case T_BYTE: return 1;
    case T_SHORT: case T_USHORT: return 2;
    case T_INT: case T_UINT: case T_FLOAT: return 4;
    case T_LONG: case T_ULONG: case T_DOUBLE: case T_TIMESPAN: case T_CORR: return 8;
    case T_GUID: case T_IPADDR: return 16;
    case T_IPEP: return 20 | CLS_PORT;
    case T_SILO: return 24 | CLS_PORT;
    case T_STRING: return 4 | CLS_STR;
    case T_GRAIN: case T_ACT: return 28 | CLS_KEY;
    case T_DATE: return 8 | CLS_DATE;
    default: return CLS_SLOW;  // char, decimal, activation address, list, nested dict, SpecifiedType, invalid
    }
}

// One header value whose token (class cls) sits at p - 1: the common-case form of skip_value, branch-free except
// for the rare classes.  The speculative reads (a length at +0 or +24, a port at +16, a DateTime at +0) are
// issued together at positions clamped into the header, and only the ones the class needs are used.
template <bool CANON = false, class S>
__device__ __forceinline__ uint32_t skip_value_fast(const S& w, typename S::P end, uint32_t cls, typename S::P& p,
                                                    bool* noncanon = nullptr) {
    using P = typename S::P;
    if (cls & CLS_SLOW) {
        p -= 1;
        return skip_value<CANON>(w, end, p, noncanon);
    }
    const P lim = end - 4;  // the header holds >= 4 bytes before p (intro + count), so lim >= 0
    auto at = [&](P q) { return q < lim ? q : lim; };
    const uint32_t r0 = ld32(w, at(p)), r4 = ld32(w, at(p + 4)), r16 = ld32(w, at(p + 16)), r20 = ld32(w, at(p + 20)),
                   r24 = ld32(w, at(p + 24));
    const P fixed = cls & CLS_SIZE;
    const bool fits = fixed <= end - p;
    const bool is_key = cls & CLS_KEY, is_str = cls & CLS_STR;
    const int32_t len = (int32_t)(is_key ? r24 : r0);
    const bool keyext = (r20 >> 24) == 6u;  // category byte of TypeCodeData (key at p: N0, N1, TCD)
    bool bad = (is_str && len < -1) || (is_key && (keyext ? len < 1 : len != -1)) || ((cls & CLS_PORT) && r16 > 65535u);
    bool unsup = false;
    if (cls & CLS_DATE) {
        const uint64_t v = (uint64_t)r0 | ((uint64_t)r4 << 32);
        unsup = (v >> 63) != 0;
        bad = bad || (v & 0x3FFFFFFFFFFFFFFFull) > kMaxTicks;
    }
    const P var = (is_str || is_key) && len > 0 ? (P)len : 0;
    const P sz = fixed + var;
    const bool fits_all = fits && var <= end - p - fixed;
    uint32_t st = !fits ? ORL_DEC_MALFORMED : unsup ? ORL_DEC_UNSUPPORTED : (bad || !fits_all) ? ORL_DEC_MALFORMED : ORL_DEC_OK;
    // KeyExt grain: the extension must not be blank (UniqueKey.cs:328-345) — rare, so a branch
    if (!st && is_key && keyext && all_whitespace(w, p + 28, var)) st = ORL_DEC_MALFORMED;
    if (CANON && !st && var > 0 && !strict_utf8(w, p + (is_key ? 28 : 4), var)) *noncanon = true;
    p += sz;
    return st;
}

// One frame's header [p, end) (frame validated by the caller) -> status + the two 16-byte halves of its record.
template <class S>
__device__ uint32_t decode_header(const S& w, typename S::P p, typename S::P end, uint32_t sender_override,
                                  const SiloAddrEntry* __restrict__ tab, const uint16_t* lut, uint4& r0, uint4& r1) {
    uint32_t st = ORL_DEC_OK;
    uint32_t cat_v = 0, cat_st = 0;           // 0 absent, 1 Int, 2 other type (cast fails)
    uint32_t ts_st = 0, ss_st = 0;            // 0 absent / null, 1 SiloAddress, 2 other type
    typename S::P ts_p = 0, ss_p = 0, tg_p = 0;
    bool tg = false, ta = false;
    // DeserializeMessageHeaders: StringObjDict, int32 count, count x (byte key, value); duplicate keys throw.
    if (5 > end - p || ld8(w, p) != T_DICT) st = ORL_DEC_MALFORMED;
    int32_t count = 0;
    if (!st) {
        count = (int32_t)ld32(w, p + 1);
        p += 5;
        if (count < 0) st = ORL_DEC_MALFORMED;
    }
    // duplicate keys: a 32-bit mask for keys < 32 (every Message.Header value); larger keys (legal bytes, never
    // written by the reference) take the rare path through a 256-bit mask
    uint32_t seen = 0;
    uint64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    for (int32_t e = 0; !st && e < count; ++e) {
        if (2 > end - p) { st = ORL_DEC_MALFORMED; break; }
        const uint32_t kt = ld32(w, p - 2) >> 16;  // key, token: p >= frame + 10, so p - 2 is in the frame
        const uint32_t key = kt & 0xFFu;
        const uint32_t tok = (kt >> 8) & 0xFFu;
        const typename S::P vp = p + 2;  // first byte after the value token
        p = vp;
        st = skip_value_fast(w, end, lut[tok], p);
        if (st) break;
        bool dup;
        if (key < 32u) {
            const uint32_t bit = 1u << key;
            dup = (seen & bit) != 0;
            seen |= bit;
        } else {
            const uint32_t q = key >> 6;
            const uint64_t bit = 1ull << (key & 63u);
            dup = ((q == 0 ? h0 : q == 1 ? h1 : q == 2 ? h2 : h3) & bit) != 0;
            h0 |= q == 0 ? bit : 0; h1 |= q == 1 ? bit : 0; h2 |= q == 2 ? bit : 0; h3 |= q == 3 ? bit : 0;
        }
        if (dup) { st = ORL_DEC_MALFORMED; break; }
        // captures, as selects
        const bool is_int = tok == T_INT, is_silo = tok == T_SILO, is_null = tok == T_NULL;
        const uint32_t sst = is_silo ? 1u : is_null ? 0u : 2u;
        if (key == H_CATEGORY) { cat_st = is_int ? 1u : 2u; cat_v = ld32(w, vp); }
        if (key == H_TARGET_SILO) { ts_st = sst; ts_p = vp; }
        if (key == H_SENDING_SILO) { ss_st = sst; ss_p = vp; }
        if (key == H_TARGET_GRAIN) { tg = tok == T_GRAIN; tg_p = vp; }
        if (key == H_TARGET_ACTIVATION) ta = tok == T_ACT;
    }
    // the getters, in the order the oracle defines (oracle/wire_codec.py decode_for_route)
    uint32_t sending = sender_override, target_silo = 0, flags = 0, aux = 0;
    uint64_t tcd = 0, n0 = 0, n1 = 0;
    if (cat_st != 1) cat_v = 0;
    if (!st && (cat_st == 2 || cat_v > 255u)) st = ORL_DEC_MALFORMED;
    if (!st && ts_st == 2) st = ORL_DEC_MALFORMED;
    if (!st && sender_override == ORL_SENDER_FROM_HEADER) {
        if (ss_st == 2) st = ORL_DEC_MALFORMED;
        else if (ss_st == 0) st = ORL_DEC_NO_SENDER;
        else if ((sending = silo_lookup(tab, w, ss_p)) == 0xFFu) st = ORL_DEC_UNKNOWN_SILO;
    }
    if (!st && !tg) st = ORL_DEC_NO_TARGET;
    if (!st) {
        n0 = ld64(w, tg_p);
        n1 = ld64(w, tg_p + 8);
        tcd = ld64(w, tg_p + 16);
        if ((tcd >> 56) == 6u) {  // KeyExt: uniform hash over Write(UniqueKey) (UniqueKey.cs:288-294)
            const uint32_t len = ld32(w, tg_p + 24);
            if (!strict_utf8(w, tg_p + 28, len)) st = ORL_DEC_UNSUPPORTED;
            else {
                aux = jenkins_stream(w, tg_p, 28u + len);
                flags |= ORL_HDR_HASH_VALID;
            }
        }
    }
    if (!st && ta && ts_st == 1) {
        if ((target_silo = silo_lookup(tab, w, ts_p)) == 0xFFu) st = ORL_DEC_UNKNOWN_SILO;
        else flags |= ORL_HDR_ADDRESS_COMPLETE;
    }
    if (st) {
        r0 = make_uint4(0, 0, 0, 0);
        r1 = make_uint4(0, 0, 0, 0);
    } else {
        r0 = make_uint4((uint32_t)tcd, (uint32_t)(tcd >> 32), (uint32_t)n0, (uint32_t)(n0 >> 32));
        r1 = make_uint4((uint32_t)n1, (uint32_t)(n1 >> 32),
                        (sending & 0xFFu) | (cat_v << 8) | (flags << 16) | ((target_silo & 0xFFu) << 24), aux);
    }
    return st;
}

// Frame prefix checks (IncomingMessageBuffer.cs:94-135): the 8-byte lengths inside the buffer, both lengths >= 0,
// header + body inside the buffer.  hl / bl are the two int32 lengths.
__device__ __forceinline__ bool frame_ok(uint64_t off, uint64_t nbytes, int32_t hl, int32_t bl) {
    return hl >= 0 && bl >= 0 && (uint64_t)hl + (uint64_t)bl <= nbytes - off - 8;
}
__device__ __forceinline__ bool prefix_in_buffer(uint64_t off, uint64_t nbytes) { return off <= nbytes && nbytes - off >= 8; }

constexpr uint32_t kDeferred = 0xFEu;  // pipelined kernel: header longer than its window, left to k_decode_deferred

// Simple form: one lane per frame, parsing straight from HBM through L1/L2 (small batches).
__global__ __launch_bounds__(256) void k_decode_frames(const uint32_t* __restrict__ buf, uint64_t nbytes,
                                                       const uint64_t* __restrict__ offs, uint32_t n, uint32_t sender_override,
                                                       const SiloAddrEntry* __restrict__ tab, uint4* __restrict__ out,
                                                       uint8_t* __restrict__ status, uint32_t* __restrict__ n_bad) {
    __shared__ uint16_t lut[256];
    lut[threadIdx.x] = (uint16_t)token_class(threadIdx.x);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t off = offs[i];
    uint4 r0 = make_uint4(0, 0, 0, 0), r1 = make_uint4(0, 0, 0, 0);
    uint32_t st = ORL_DEC_MALFORMED;
    if (prefix_in_buffer(off, nbytes)) {
        const GlobalSrc pre{buf, (off + 7) >> 2};
        const int32_t hl = (int32_t)ld32(pre, off), bl = (int32_t)ld32(pre, off + 4);
        if (frame_ok(off, nbytes, hl, bl)) {
            const uint64_t end = off + 8 + (uint64_t)hl;
            st = decode_header(GlobalSrc{buf, (end - 1) >> 2}, off + 8, end, sender_override, tab, lut, r0, r1);
        }
    }
    if (st && n_bad) atomicAdd(n_bad, 1u);
    out[2ull * i] = r0;
    out[2ull * i + 1] = r1;
    status[i] = (uint8_t)st;
}

// Fallback for the frames the pipelined kernel could not finish (a header longer than kHeldWords words, or more
// than 64 long headers in one wave's share): a no-op unless the kernel raised *any_deferred.  Each wave ballots
// its 64 statuses; for every deferred frame the whole wave copies the frame (prefix + header, up to kLongWords words)
// into the wave's LDS buffer with coalesced loads, and that frame's lane parses it from LDS.  Headers beyond
// kLongWords words are parsed from HBM.
constexpr uint32_t kLongWords = 1024;

__global__ __launch_bounds__(256) void k_decode_deferred(const uint32_t* __restrict__ buf, uint64_t nbytes,
                                                         const uint64_t* __restrict__ offs, uint32_t n, uint32_t sender_override,
                                                         const SiloAddrEntry* __restrict__ tab, uint4* __restrict__ out,
                                                         uint8_t* __restrict__ status, uint32_t* __restrict__ n_bad,
                                                         const uint32_t* __restrict__ any_deferred) {
    if (*any_deferred == 0) return;  // the pipelined kernel finished every frame itself
    __shared__ uint32_t big[4][kLongWords];
    __shared__ uint16_t lut[256];
    lut[threadIdx.x] = (uint16_t)token_class(threadIdx.x);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool mine = i < n && status[i] == kDeferred;
    uint64_t todo = __ballot(mine);
    if (!todo) return;  // wave-uniform; no block barrier follows
    const uint64_t off = mine ? offs[i] : 0;
    const int32_t hl = mine ? (int32_t)ld32(GlobalSrc{buf, (off + 7) >> 2}, off) : 0;  // validated by the pipelined kernel
    const uint32_t w_lo = (uint32_t)(off >> 2), w_hi = (uint32_t)(off >> 34);
    const uint32_t words = (uint32_t)(((off & 3u) + 8u + (uint64_t)hl + 3u) / 4u);
    uint32_t* row = big[wv];
    while (todo) {
        const uint32_t j = (uint32_t)__builtin_ctzll(todo);
        todo &= todo - 1;
        const uint32_t nw = (uint32_t)__builtin_amdgcn_readlane(words, j);
        if (nw <= kLongWords) {
            const uint64_t w0 = (uint64_t)__builtin_amdgcn_readlane(w_lo, j) | ((uint64_t)__builtin_amdgcn_readlane(w_hi, j) << 32);
            for (uint32_t k = lane; k < nw; k += 64) row[k] = buf[w0 + k];
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == j) {
            uint4 r0 = make_uint4(0, 0, 0, 0), r1 = make_uint4(0, 0, 0, 0);
            uint32_t st;
            const uint32_t q0 = (uint32_t)(off & 3u);
            if (nw <= kLongWords)
                st = decode_header(LdsSrc{row}, q0 + 8, q0 + 8 + (uint32_t)hl, sender_override, tab, lut, r0, r1);
            else
                st = decode_header(GlobalSrc{buf, (off + 7 + (uint64_t)hl) >> 2}, off + 8, off + 8 + (uint64_t)hl, sender_override,
                                   tab, lut, r0, r1);
            if (st && n_bad) atomicAdd(n_bad, 1u);
            out[2ull * i] = r0;
            out[2ull * i + 1] = r1;
            status[i] = (uint8_t)st;
        }
        __builtin_amdgcn_wave_barrier();  // the buffer is rewritten for the next frame
    }
}

// Pipelined form.  A persistent wave walks 64-frame chunks.  For every frame of a chunk it loads the 64-word
// (256-byte) window that starts at the frame's first aligned word — one coalesced load per frame, issued for the
// NEXT chunk while the current chunk is parsed, so the HBM latency hides behind the parse — then copies the
// window into the frame's LDS row and parses it there with 32-bit positions: one pass over the header bytes
// instead of the dozens of L2 requests per frame that lanes parsing 64 different frames through a 32-KB L1 cost.
// Rows are 65 words apart, so lanes reading the same relative word hit distinct banks.  Window loads are
// clamped to the buffer's last word.  A header that does not fit its window is held in a per-wave list and, after
// the wave's last chunk, parsed 16 at a time from kHeldWords-word LDS rows; beyond that it is left to
// k_decode_deferred (status kDeferred, *any_deferred = 1).
constexpr uint32_t kRowWords = 64;
constexpr uint32_t kRowStride = kRowWords + 1;
constexpr uint32_t kHeldWords = 64 * kRowStride / 16;  // 260 words per held frame, 16 at a time
constexpr uint32_t kHeldMax = 64;
constexpr size_t kPipeMinFrames = 1u << 16;  // below this the simple form fills the chip better

__device__ __forceinline__ void load_windows(const uint32_t* __restrict__ buf, uint64_t last_word, uint64_t off,
                                             uint32_t lane, uint32_t (&v)[64]) {
    const uint32_t w_lo = (uint32_t)(off >> 2), w_hi = (uint32_t)(off >> 34);
#pragma unroll
    for (uint32_t j = 0; j < 64; ++j) {
        // frame j's first word, broadcast from lane j into scalar registers
        const uint64_t w0 = (uint64_t)__builtin_amdgcn_readlane(w_lo, j) | ((uint64_t)__builtin_amdgcn_readlane(w_hi, j) << 32);
        const uint64_t wi = w0 + lane;
        v[j] = buf[wi < last_word ? wi : last_word];
    }
}

__global__ __launch_bounds__(256) void k_decode_frames_pipe(const uint32_t* __restrict__ buf, uint64_t nbytes,
                                                            const uint64_t* __restrict__ offs, uint32_t n,
                                                            uint32_t sender_override, const SiloAddrEntry* __restrict__ tab,
                                                            uint4* __restrict__ out, uint8_t* __restrict__ status,
                                                            uint32_t* __restrict__ n_bad, uint32_t* __restrict__ any_deferred) {
    __shared__ uint32_t rows[4][64 * kRowStride];
    __shared__ uint32_t held[4][kHeldMax];
    __shared__ uint32_t n_held[4];
    __shared__ uint16_t lut[256];
    lut[threadIdx.x] = (uint16_t)token_class(threadIdx.x);
    if ((threadIdx.x & 63u) == 0) n_held[threadIdx.x >> 6] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t n_chunks = (n + 63) / 64;
    const uint32_t stride = gridDim.x * 4;
    uint32_t c = blockIdx.x * 4 + wv;
    if (c >= n_chunks) return;  // wave-uniform: the kernel has no block-wide barrier after this point
    const uint64_t last_word = (nbytes + 3) / 4 - 1;  // launcher guarantees nbytes >= 8
    uint32_t* my = rows[wv];
    const LdsSrc l{my + lane * kRowStride};
    auto frame_off = [&](uint32_t chunk) -> uint64_t {
        const uint32_t i = chunk * 64 + lane;
        return chunk < n_chunks && i < n ? offs[i] : ~0ull;
    };
    auto finish = [&](uint32_t i, uint32_t st, const uint4& r0, const uint4& r1) {
        if (st == kDeferred) {
            *any_deferred = 1u;
        } else {
            if (st && n_bad) atomicAdd(n_bad, 1u);
            out[2ull * i] = r0;
            out[2ull * i + 1] = r1;
        }
        status[i] = (uint8_t)st;
    };
    uint64_t off = frame_off(c);
    uint32_t v[64];
    load_windows(buf, last_word, off == ~0ull ? 0 : off, lane, v);
    uint64_t off_next = frame_off(c + stride);
    while (true) {
#pragma unroll
        for (uint32_t j = 0; j < 64; ++j) my[j * kRowStride + lane] = v[j];
        const uint32_t cn = c + stride;
        const uint64_t off_nn = frame_off(cn + stride);
        if (cn < n_chunks) load_windows(buf, last_word, off_next == ~0ull ? 0 : off_next, lane, v);
        __builtin_amdgcn_wave_barrier();
        const uint32_t i = c * 64 + lane;
        if (i < n) {
            uint4 r0 = make_uint4(0, 0, 0, 0), r1 = make_uint4(0, 0, 0, 0);
            uint32_t st = ORL_DEC_MALFORMED;
            bool hold = false;
            if (prefix_in_buffer(off, nbytes)) {
                const uint32_t q0 = (uint32_t)(off & 3u);  // the frame's first byte in its row
                const int32_t hl = (int32_t)ld32(l, q0), bl = (int32_t)ld32(l, q0 + 4);
                if (frame_ok(off, nbytes, hl, bl)) {
                    if ((uint64_t)hl <= kRowWords * 4 - 8 - q0) {
                        st = decode_header(l, q0 + 8, q0 + 8 + (uint32_t)hl, sender_override, tab, lut, r0, r1);
                    } else {
                        const uint32_t k = atomicAdd(&n_held[wv], 1u);
                        if (k < kHeldMax) { held[wv][k] = i; hold = true; }
                        else st = kDeferred;
                    }
                }
            }
            if (!hold) finish(i, st, r0, r1);
        }
        if (cn >= n_chunks) break;
        __builtin_amdgcn_wave_barrier();  // the rows are rewritten next iteration
        c = cn;
        off = off_next;
        off_next = off_nn;
    }
    // the held long headers, 16 at a time
    __builtin_amdgcn_wave_barrier();
    const uint32_t nh = min(n_held[wv], kHeldMax);
    for (uint32_t b = 0; b < nh; b += 16) {
        const uint32_t m = min(16u, nh - b);
        const bool act = lane < m;
        const uint32_t fi = act ? held[wv][b + lane] : 0;
        const uint64_t foff = act ? offs[fi] : 0;
        const int32_t fhl = act ? (int32_t)ld32(GlobalSrc{buf, (foff + 7) >> 2}, foff) : 0;  // checked in the loop
        const uint32_t fw = (uint32_t)(((foff & 3u) + 8u + (uint64_t)fhl + 3u) / 4u);
        const uint32_t w_lo = (uint32_t)(foff >> 2), w_hi = (uint32_t)(foff >> 34);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t k = 0; k < m; ++k) {
            const uint32_t nw = (uint32_t)__builtin_amdgcn_readlane(fw, k);
            if (nw > kHeldWords) continue;
            const uint64_t w0 = (uint64_t)__builtin_amdgcn_readlane(w_lo, k) | ((uint64_t)__builtin_amdgcn_readlane(w_hi, k) << 32);
            for (uint32_t t = lane; t < nw; t += 64) my[k * kHeldWords + t] = buf[w0 + t];
        }
        __builtin_amdgcn_wave_barrier();
        if (act) {
            uint4 r0 = make_uint4(0, 0, 0, 0), r1 = make_uint4(0, 0, 0, 0);
            uint32_t st = kDeferred;
            if (fw <= kHeldWords) {
                const uint32_t q0 = (uint32_t)(foff & 3u);
                st = decode_header(LdsSrc{my + lane * kHeldWords}, q0 + 8, q0 + 8 + (uint32_t)fhl, sender_override, tab, lut, r0, r1);
            }
            finish(fi, st, r0, r1);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- f2 emit: SetTargetPlacement on routed frames (orl_stamp_frames_device) ----------------------------------
// Message.SetTargetPlacement (Message.cs:1079-1096) on the header dictionary DeserializeMessageHeaders built
// (entries in wire order, no free slots), then SerializeMessageHeaders: PRIOR_MESSAGE_ID / _TIMES removed on a new
// placement or an activation change (Dictionary.Remove pushes the entry on a LIFO free list), TARGET_ACTIVATION
// and TARGET_SILO set (an existing key keeps its position; a new key takes the free-list head, else is appended),
// and on a new placement IS_NEW_PLACEMENT = true and NEW_GRAIN_TYPE.  The oracle is wire_codec.stamp_frame.
enum : uint32_t { H_NEW_GRAIN_TYPE = 11, H_IS_NEW_PLACEMENT = 21, H_PRIOR_ID = 28, H_PRIOR_TIMES = 29 };
enum : uint32_t { NE_KEEP = 0, NE_REMOVE = 1, NE_ACT = 2, NE_SILO = 3, NE_ISNEW = 4, NE_GTYPE = 5 };
constexpr uint32_t kSpecials = 6;  // 28, 29, 22, 24, 21, 11

struct StampPlan {
    uint32_t st;
    uint64_t hdr, end;      // header start / end (absolute)
    uint64_t dict_end;      // one past the dictionary's last byte (bytes after it are not re-serialized)
    uint64_t hl_new;        // new header length
    int32_t count_new;
    // the special entries present in the header: [start, end) of the whole entry (key byte .. value end)
    uint64_t s_start[kSpecials], s_end[kSpecials];
    uint32_t present;       // bit k: special k present
    uint32_t kind[kSpecials];
    uint32_t app;           // appended kinds, 4 bits each, first in the low nibble
    uint32_t n_app;
    uint64_t act_tcd, act_n0, act_n1;
    uint32_t host, gt_off, gt_len;
};

__device__ __forceinline__ uint32_t special_index(uint32_t key) {
    return key == H_PRIOR_ID ? 0u : key == H_PRIOR_TIMES ? 1u : key == H_TARGET_ACTIVATION ? 2u
         : key == H_TARGET_SILO ? 3u : key == H_IS_NEW_PLACEMENT ? 4u : key == H_NEW_GRAIN_TYPE ? 5u : kSpecials;
}

__device__ __forceinline__ uint32_t new_entry_len(uint32_t kind, uint32_t gt_len) {
    return kind == NE_ACT ? 30u : kind == NE_SILO ? 26u : kind == NE_ISNEW ? 2u : kind == NE_GTYPE ? 6u + gt_len : 0u;
}

__device__ bool grain_type_lookup(const GrainTypeEntry* __restrict__ gt, uint32_t code, uint32_t& off, uint32_t& len) {
    uint32_t s = fmix32(code) & (kGrainTypeSlots - 1u);
    for (uint32_t probe = 0; probe < kGrainTypeSlots; ++probe) {
        const GrainTypeEntry e = gt[s];
        if (!e.used) return false;
        if ((uint32_t)e.code == code) { off = e.off; len = e.len; return true; }
        s = (s + 1u) & (kGrainTypeSlots - 1u);
    }
    return false;
}

// One frame's header [hdr, end) (prefix already validated) -> plan.  Statuses in the order of
// wire_codec.stamp_frames.
template <class S>
__device__ StampPlan stamp_plan(const S& w, typename S::P hdr, typename S::P end, uint32_t route, uint32_t act, uint64_t i,
                                const orl_grain_key* __restrict__ act_keys, uint32_t n_act_keys,
                                const orl_grain_key* __restrict__ new_act_keys, const GrainTypeEntry* __restrict__ gt,
                                const uint32_t* __restrict__ silo_words, const uint16_t* lut) {
    using P_t = typename S::P;
    StampPlan P;
    P.st = ORL_STAMP_MALFORMED;
    P.present = 0;
#pragma unroll
    for (uint32_t j = 0; j < kSpecials; ++j) P.s_start[j] = P.s_end[j] = 0;
    P.app = 0;
    P.n_app = 0;
    P.hdr = hdr;
    P.end = end;
    P.hl_new = end - hdr;
    P.count_new = 0;
    // structural parse (DeserializeMessageHeaders), recording the special entries
    P_t p = hdr;
    uint32_t st = ORL_DEC_OK;
    bool noncanon = false;
    uint32_t tok22 = 0;
    P_t v22 = 0;
    int32_t count = 0;
    if (5 > end - p || ld8(w, p) != T_DICT) st = ORL_DEC_MALFORMED;
    if (!st) {
        count = (int32_t)ld32(w, p + 1);
        p += 5;
        if (count < 0) st = ORL_DEC_MALFORMED;
    }
    uint32_t seen = 0;
    uint64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    for (int32_t e = 0; !st && e < count; ++e) {
        if (2 > end - p) { st = ORL_DEC_MALFORMED; break; }
        const P_t es = p;
        const uint32_t kt = ld32(w, p - 2) >> 16;  // key, token: p >= frame + 10
        const uint32_t key = kt & 0xFFu, tok = (kt >> 8) & 0xFFu;
        p += 2;
        st = skip_value_fast<true>(w, end, lut[tok], p, &noncanon);
        if (st) break;
        bool dup;
        if (key < 32u) {
            dup = (seen >> key) & 1u;
            seen |= 1u << key;
        } else {
            const uint32_t q = key >> 6;
            const uint64_t bit = 1ull << (key & 63u);
            dup = ((q == 0 ? h0 : q == 1 ? h1 : q == 2 ? h2 : h3) & bit) != 0;
            h0 |= q == 0 ? bit : 0; h1 |= q == 1 ? bit : 0; h2 |= q == 2 ? bit : 0; h3 |= q == 3 ? bit : 0;
        }
        if (dup) { st = ORL_DEC_MALFORMED; break; }
        const uint32_t k = special_index(key);
        if (k < kSpecials) {  // unrolled: the struct's arrays stay in registers
            P.present |= 1u << k;
#pragma unroll
            for (uint32_t j = 0; j < kSpecials; ++j) {
                P.s_start[j] = j == k ? es : P.s_start[j];
                P.s_end[j] = j == k ? p : P.s_end[j];
            }
            if (k == 2) { tok22 = tok; v22 = es + 2; }
        }
    }
    if (st) {
        P.st = st == ORL_DEC_UNSUPPORTED ? ORL_STAMP_UNSUPPORTED : ORL_STAMP_MALFORMED;
        return P;
    }
    P.dict_end = p;
    const uint32_t rst = (route >> 16) & 0xFFu;
    if (rst == ORL_ST_ADDRESS_COMPLETE) { P.st = ORL_STAMP_COMPLETE; return P; }
    if (rst != ORL_ST_HIT && rst != ORL_ST_NEW_PLACEMENT) { P.st = ORL_STAMP_SKIPPED; return P; }
    if (noncanon) { P.st = ORL_STAMP_UNSUPPORTED; return P; }
    const bool np = rst == ORL_ST_NEW_PLACEMENT;
    P.host = (route >> 8) & 0xFFu;
    P.gt_off = P.gt_len = 0;
    {   // the host silo's address must be known (orl_silo_address_set); SiloAddress.Zero never is a silo
        uint32_t any = 0;
        for (uint32_t k = 0; k < 6; ++k) any |= silo_words[P.host * 6 + k];
        if (!any) { P.st = ORL_STAMP_UNSUPPORTED; return P; }
    }
    if (np) {
        // SpecifyCreation(silo, strategy, context.GetGrainTypeName(grain)): the target's type code
        // (TARGET_GRAIN was parsed above; routing needs it, so it is a GrainId here)
        uint32_t code = 0;
        // find TARGET_GRAIN again: it is not a special entry; scan for it (rare path: new placements)
        P_t q = hdr + 5;
        bool found = false;
        for (int32_t e = 0; e < count; ++e) {
            const uint32_t key = ld8(w, q), tok = ld8(w, q + 1);
            if (key == H_TARGET_GRAIN && tok == T_GRAIN) { code = ld32(w, q + 2 + 16); found = true; break; }
            q += 2;
            (void)skip_value_fast(w, end, lut[tok], q);
        }
        if (!found || !grain_type_lookup(gt, code, P.gt_off, P.gt_len)) { P.st = ORL_STAMP_UNSUPPORTED; return P; }
        if (!new_act_keys) { P.st = ORL_STAMP_UNSUPPORTED; return P; }
        const orl_grain_key a = new_act_keys[i];
        P.act_tcd = a.type_code_data; P.act_n0 = a.n0; P.act_n1 = a.n1;
    } else {
        if (act >= n_act_keys) { P.st = ORL_STAMP_UNSUPPORTED; return P; }
        const orl_grain_key a = act_keys[act];
        P.act_tcd = a.type_code_data; P.act_n0 = a.n0; P.act_n1 = a.n1;
    }
    bool differs = false;
    if (P.present & 4u) {
        if (tok22 != T_ACT) { P.st = ORL_STAMP_MALFORMED; return P; }  // null.Equals(...) in SetTargetPlacement
        differs = ld64(w, v22) != P.act_n0 || ld64(w, v22 + 8) != P.act_n1 || ld64(w, v22 + 16) != P.act_tcd ||
                  (int32_t)ld32(w, v22 + 24) != -1;
    }
    // the dictionary updates
#pragma unroll
    for (uint32_t k = 0; k < kSpecials; ++k) P.kind[k] = NE_KEEP;
    uint32_t fstack = 0, nfree = 0;  // free-list: entry indices 0 (PRIOR_ID) / 1 (PRIOR_TIMES), top = last pushed
    int32_t cnt = count;
    if (np || differs) {
        if (P.present & 1u) { P.kind[0] = NE_REMOVE; fstack = (fstack << 2) | 0u; ++nfree; --cnt; }
        if (P.present & 2u) { P.kind[1] = NE_REMOVE; fstack = (fstack << 2) | 1u; ++nfree; --cnt; }
        // (the free list holds at most these two; its head is the last removed)
    }
    auto set = [&](uint32_t k, uint32_t kind) {
        if (P.present & (1u << k)) { P.kind[k] = kind; return; }
        ++cnt;
        if (nfree) {
            if ((fstack & 3u) == 0) P.kind[0] = kind;
            else P.kind[1] = kind;
            fstack >>= 2;
            --nfree;
            return;
        }
        P.app |= kind << (4u * P.n_app);
        ++P.n_app;
    };
    set(2, NE_ACT);
    set(3, NE_SILO);
    if (np) {
        set(4, NE_ISNEW);
        set(5, NE_GTYPE);
    }
    // new header length
    int64_t hl_new = (int64_t)(P.dict_end - P.hdr);
    (void)P_t(0);
#pragma unroll
    for (uint32_t k = 0; k < kSpecials; ++k)
        if ((P.present >> k) & 1u && P.kind[k] != NE_KEEP)
            hl_new += (int64_t)new_entry_len(P.kind[k], P.gt_len) - (int64_t)(P.s_end[k] - P.s_start[k]);
    for (uint32_t a = 0; a < P.n_app; ++a) hl_new += new_entry_len((P.app >> (4u * a)) & 15u, P.gt_len);
    P.hl_new = (uint64_t)hl_new;
    P.count_new = cnt;
    P.st = ORL_STAMP_OK;
    return P;
}

// Output words of one frame.  The frame's output starts 4-byte aligned and owns its words up to its aligned end.
struct WordWriter {
    uint32_t* dst;
    uint64_t acc = 0;
    uint32_t nacc = 0;  // bytes pending in acc (0..3)
    __device__ __forceinline__ void put32(uint32_t v) {
        acc |= (uint64_t)v << (8u * nacc);
        *dst++ = (uint32_t)acc;
        acc >>= 32;
    }
    __device__ __forceinline__ void put8(uint32_t b) {
        acc |= (uint64_t)(b & 0xFFu) << (8u * nacc);
        if (++nacc == 4) { *dst++ = (uint32_t)acc; acc = 0; nacc = 0; }
    }
    __device__ __forceinline__ void put64(uint64_t v) { put32((uint32_t)v); put32((uint32_t)(v >> 32)); }
    __device__ __forceinline__ void flush() { if (nacc) *dst++ = (uint32_t)acc; }
    template <class S>
    __device__ void copy(const S& s, typename S::P p, typename S::P len) {
        for (; len >= 32; len -= 32, p += 32) {  // eight words in flight before the first store
            uint32_t v[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) v[k] = ld32(s, p + 4 * k);
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) put32(v[k]);
        }
        for (; len >= 4; len -= 4, p += 4) put32(ld32(s, p));
        for (; len; --len, ++p) put8(ld8(s, p));
    }
};

__device__ void emit_entry(WordWriter& o, uint32_t kind, const StampPlan& P, const uint32_t* __restrict__ silo_words,
                           const uint8_t* __restrict__ gt_blob) {
    switch (kind) {
    case NE_ACT:
        o.put8(H_TARGET_ACTIVATION); o.put8(T_ACT);
        o.put64(P.act_n0); o.put64(P.act_n1); o.put64(P.act_tcd); o.put32(0xFFFFFFFFu);
        break;
    case NE_SILO:
        o.put8(H_TARGET_SILO); o.put8(T_SILO);
        for (uint32_t k = 0; k < 6; ++k) o.put32(silo_words[P.host * 6 + k]);
        break;
    case NE_ISNEW:
        o.put8(H_IS_NEW_PLACEMENT); o.put8(T_TRUE);
        break;
    case NE_GTYPE:
        o.put8(H_NEW_GRAIN_TYPE); o.put8(T_STRING); o.put32(P.gt_len);
        for (uint32_t k = 0; k < P.gt_len; ++k) o.put8(gt_blob[P.gt_off + k]);
        break;
    default: break;
    }
}

// The stamped frame: prefix, dictionary with the special entries replaced / removed and the new ones appended,
// then the body (copied from HBM at body_pos).
template <class S>
__device__ void write_stamped(WordWriter& wr, const S& w, const StampPlan& P, const GlobalSrc& g, uint64_t body_pos,
                              uint64_t bl, const uint32_t* __restrict__ silo_words, const uint8_t* __restrict__ gt_blob) {
    using P_t = typename S::P;
    wr.put32((uint32_t)P.hl_new);
    wr.put32((uint32_t)bl);
    wr.put8(T_DICT);
    wr.put32((uint32_t)P.count_new);
    uint64_t pos = P.hdr + 5;
    while (true) {  // the next special entry at or after pos (selects only: no dynamic indexing)
        uint64_t ns = ~0ull, ne = 0;
        uint32_t nkind = NE_KEEP;
#pragma unroll
        for (uint32_t k = 0; k < kSpecials; ++k) {
            const bool take = ((P.present >> k) & 1u) && P.s_start[k] >= pos && P.s_start[k] < ns;
            ns = take ? P.s_start[k] : ns;
            ne = take ? P.s_end[k] : ne;
            nkind = take ? P.kind[k] : nkind;
        }
        if (ns == ~0ull) break;
        wr.copy(w, (P_t)pos, (P_t)(ns - pos));
        if (nkind == NE_KEEP) wr.copy(w, (P_t)ns, (P_t)(ne - ns));
        else emit_entry(wr, nkind, P, silo_words, gt_blob);
        pos = ne;
    }
    wr.copy(w, (P_t)pos, (P_t)(P.dict_end - pos));
    for (uint32_t a = 0; a < P.n_app; ++a) emit_entry(wr, (P.app >> (4u * a)) & 15u, P, silo_words, gt_blob);
    wr.copy(g, body_pos, bl);
    wr.flush();
}

// Size (WRITE = false) and write passes for one frame whose prefix is (hl, bl) at off, parsed from w at hdr.
template <bool WRITE, class S>
__device__ __forceinline__ void stamp_one(const S& w, typename S::P hdr, uint32_t i, uint64_t off, int32_t hl, int32_t bl,
                                          const uint32_t* __restrict__ buf, const uint32_t* __restrict__ route,
                                          const uint32_t* __restrict__ act, const orl_grain_key* __restrict__ act_keys,
                                          uint32_t n_act_keys, const orl_grain_key* __restrict__ new_act_keys,
                                          const GrainTypeEntry* __restrict__ gt, const uint8_t* __restrict__ gt_blob,
                                          const uint32_t* __restrict__ silo_words, uint64_t* __restrict__ sizes,
                                          const uint64_t* __restrict__ out_offs, uint32_t* __restrict__ out, uint64_t out_cap,
                                          uint8_t* __restrict__ status, const uint16_t* lut) {
    const StampPlan P = stamp_plan(w, hdr, hdr + (typename S::P)hl, route[i], act[i], i, act_keys, n_act_keys, new_act_keys,
                                   gt, silo_words, lut);
    const uint64_t size = 8 + (P.st == ORL_STAMP_OK ? P.hl_new : (uint64_t)hl) + (uint64_t)bl;
    if (!WRITE) {
        sizes[i] = (size + 3) & ~3ull;
        return;
    }
    uint32_t st = P.st;
    const uint64_t o = out_offs[i], asz = (size + 3) & ~3ull;
    if (o > out_cap || asz > out_cap - o) st = ORL_STAMP_OVERFLOW;
    status[i] = (uint8_t)st;
    if (st == ORL_STAMP_OVERFLOW) return;
    const GlobalSrc g{buf, (off + 8 + (uint64_t)hl + (uint64_t)bl + 3) / 4 - 1};
    WordWriter wr{out + o / 4};
    if (P.st != ORL_STAMP_OK) {  // unchanged copy
        wr.copy(g, off, size);
        wr.flush();
        return;
    }
    write_stamped(wr, w, P, g, off + 8 + (uint64_t)hl, (uint64_t)bl, silo_words, gt_blob);
}

// Simple form (small batches, and the frames the pipelined form defers when *any_deferred): one lane per frame
// parsing from HBM.  An invalid prefix emits nothing.
template <bool WRITE, bool DEFERRED>
__global__ __launch_bounds__(256) void k_stamp(const uint32_t* __restrict__ buf, uint64_t nbytes, const uint64_t* __restrict__ offs,
                                               uint32_t n, const uint32_t* __restrict__ route, const uint32_t* __restrict__ act,
                                               const orl_grain_key* __restrict__ act_keys, uint32_t n_act_keys,
                                               const orl_grain_key* __restrict__ new_act_keys, const GrainTypeEntry* __restrict__ gt,
                                               const uint8_t* __restrict__ gt_blob, const uint32_t* __restrict__ silo_words,
                                               uint64_t* __restrict__ sizes, const uint64_t* __restrict__ out_offs,
                                               uint32_t* __restrict__ out, uint64_t out_cap, uint8_t* __restrict__ status,
                                               const uint32_t* __restrict__ any_deferred) {
    if (DEFERRED && *any_deferred == 0) return;
    __shared__ uint16_t lut[256];
    lut[threadIdx.x] = (uint16_t)token_class(threadIdx.x);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (DEFERRED && status[i] != kDeferred) return;
    const uint64_t off = offs[i];
    int32_t hl = -1, bl = -1;
    if (prefix_in_buffer(off, nbytes)) {
        const GlobalSrc pre{buf, (off + 7) >> 2};
        hl = (int32_t)ld32(pre, off);
        bl = (int32_t)ld32(pre, off + 4);
    }
    if (!prefix_in_buffer(off, nbytes) || !frame_ok(off, nbytes, hl, bl)) {
        if (WRITE) status[i] = ORL_STAMP_MALFORMED;
        else sizes[i] = 0;
        return;
    }
    const uint64_t end = off + 8 + (uint64_t)hl;
    stamp_one<WRITE>(GlobalSrc{buf, (end - 1) >> 2}, off + 8, i, off, hl, bl, buf, route, act, act_keys, n_act_keys,
                     new_act_keys, gt, gt_blob, silo_words, sizes, out_offs, out, out_cap, status, lut);
}

// Pipelined form (the decoder's k_decode_frames_pipe scheme): persistent waves stage every frame's 256-byte
// header window in LDS, prefetching the next chunk's windows during the current chunk, and plan / write from LDS
// with 32-bit positions; frames whose header does not fit are left to k_stamp<., true> (status kDeferred in the
// size pass, *any_deferred = 1).  Outputs are written per lane (4-byte aligned frame starts).
template <bool WRITE>
__global__ __launch_bounds__(256) void k_stamp_pipe(const uint32_t* __restrict__ buf, uint64_t nbytes,
                                                    const uint64_t* __restrict__ offs, uint32_t n, const uint32_t* __restrict__ route,
                                                    const uint32_t* __restrict__ act, const orl_grain_key* __restrict__ act_keys,
                                                    uint32_t n_act_keys, const orl_grain_key* __restrict__ new_act_keys,
                                                    const GrainTypeEntry* __restrict__ gt, const uint8_t* __restrict__ gt_blob,
                                                    const uint32_t* __restrict__ silo_words, uint64_t* __restrict__ sizes,
                                                    const uint64_t* __restrict__ out_offs, uint32_t* __restrict__ out,
                                                    uint64_t out_cap, uint8_t* __restrict__ status, uint32_t* __restrict__ any_deferred) {
    __shared__ uint32_t rows[4][64 * kRowStride];
    __shared__ uint32_t held[4][kHeldMax];
    __shared__ uint32_t n_held[4];
    __shared__ uint16_t lut[256];
    lut[threadIdx.x] = (uint16_t)token_class(threadIdx.x);
    if ((threadIdx.x & 63u) == 0) n_held[threadIdx.x >> 6] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t n_chunks = (n + 63) / 64;
    const uint32_t stride = gridDim.x * 4;
    uint32_t c = blockIdx.x * 4 + wv;
    if (c >= n_chunks) return;  // wave-uniform; no block barrier follows
    const uint64_t last_word = (nbytes + 3) / 4 - 1;  // launcher guarantees nbytes >= 8
    uint32_t* my = rows[wv];
    const LdsSrc l{my + lane * kRowStride};
    auto frame_off = [&](uint32_t chunk) -> uint64_t {
        const uint32_t i = chunk * 64 + lane;
        return chunk < n_chunks && i < n ? offs[i] : ~0ull;
    };
    uint64_t off = frame_off(c);
    uint32_t v[64];
    load_windows(buf, last_word, off == ~0ull ? 0 : off, lane, v);
    uint64_t off_next = frame_off(c + stride);
    while (true) {
#pragma unroll
        for (uint32_t j = 0; j < 64; ++j) my[j * kRowStride + lane] = v[j];
        const uint32_t cn = c + stride;
        const uint64_t off_nn = frame_off(cn + stride);
        if (cn < n_chunks) load_windows(buf, last_word, off_next == ~0ull ? 0 : off_next, lane, v);
        __builtin_amdgcn_wave_barrier();
        const uint32_t i = c * 64 + lane;
        if (i < n) {
            if (!prefix_in_buffer(off, nbytes)) {
                if (WRITE) status[i] = ORL_STAMP_MALFORMED;
                else sizes[i] = 0;
            } else {
                const uint32_t q0 = (uint32_t)(off & 3u);
                const int32_t hl = (int32_t)ld32(l, q0), bl = (int32_t)ld32(l, q0 + 4);
                if (!frame_ok(off, nbytes, hl, bl)) {
                    if (WRITE) status[i] = ORL_STAMP_MALFORMED;
                    else sizes[i] = 0;
                } else if ((uint64_t)hl > kRowWords * 4 - 8 - q0) {
                    const uint32_t k = atomicAdd(&n_held[wv], 1u);
                    if (k < kHeldMax) {
                        held[wv][k] = i;
                    } else if (!WRITE) {  // left to k_stamp<., true>
                        status[i] = kDeferred;
                        *any_deferred = 1u;
                    }
                } else {
                    if (!WRITE) status[i] = 0;
                    stamp_one<WRITE>(l, q0 + 8, i, off, hl, bl, buf, route, act, act_keys, n_act_keys, new_act_keys, gt,
                                     gt_blob, silo_words, sizes, out_offs, out, out_cap, status, lut);
                }
            }
        }
        if (cn >= n_chunks) break;
        __builtin_amdgcn_wave_barrier();  // the rows are rewritten next iteration
        c = cn;
        off = off_next;
        off_next = off_nn;
    }
    // the held long headers, 16 at a time from kHeldWords-word rows (the same frames in both passes: the
    // held / deferred split depends only on the frame and its chunk's wave)
    __builtin_amdgcn_wave_barrier();
    const uint32_t nh = min(n_held[wv], kHeldMax);
    for (uint32_t b = 0; b < nh; b += 16) {
        const uint32_t m = min(16u, nh - b);
        const bool act_ = lane < m;
        const uint32_t fi = act_ ? held[wv][b + lane] : 0;
        const uint64_t foff = act_ ? offs[fi] : 0;
        const GlobalSrc pre{buf, (foff + 7) >> 2};
        const int32_t fhl = act_ ? (int32_t)ld32(pre, foff) : 0, fbl = act_ ? (int32_t)ld32(pre, foff + 4) : 0;
        const uint32_t fw = (uint32_t)(((foff & 3u) + 8u + (uint64_t)fhl + 3u) / 4u);
        const uint32_t w_lo = (uint32_t)(foff >> 2), w_hi = (uint32_t)(foff >> 34);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t k = 0; k < m; ++k) {
            const uint32_t nw = (uint32_t)__builtin_amdgcn_readlane(fw, k);
            if (nw > kHeldWords) continue;
            const uint64_t w0 = (uint64_t)__builtin_amdgcn_readlane(w_lo, k) | ((uint64_t)__builtin_amdgcn_readlane(w_hi, k) << 32);
            for (uint32_t t = lane; t < nw; t += 64) my[k * kHeldWords + t] = buf[w0 + t];
        }
        __builtin_amdgcn_wave_barrier();
        if (act_) {
            if (fw <= kHeldWords) {
                if (!WRITE) status[fi] = 0;
                stamp_one<WRITE>(LdsSrc{my + lane * kHeldWords}, (uint32_t)(foff & 3u) + 8, fi, foff, fhl, fbl, buf, route, act,
                                 act_keys, n_act_keys, new_act_keys, gt, gt_blob, silo_words, sizes, out_offs, out, out_cap,
                                 status, lut);
            } else if (!WRITE) {
                status[fi] = kDeferred;
                *any_deferred = 1u;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__global__ void k_stamp_total(const uint64_t* __restrict__ sizes, const uint64_t* __restrict__ offs, uint32_t n,
                              uint64_t* __restrict__ total) {
    *total = n ? offs[n - 1] + sizes[n - 1] : 0;
}

}  // namespace

int launch_decode_frames(const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_offsets, size_t n,
                         uint32_t sender_override, const SiloAddrEntry* d_silo_tab, orl_msg_hdr* d_out,
                         uint8_t* d_status, uint32_t* d_n_bad, uint32_t* d_flag, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (d_n_bad) {
        const hipError_t e = hipMemsetAsync(d_n_bad, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return (int)e;
    }
    if (n == 0) return 0;
    const dim3 grid((uint32_t)((n + 255) / 256));
    if (n >= kPipeMinFrames && nbytes >= 8) {
        // persistent: 2 workgroups (66.5 KB LDS each) per CU; then the deferred long headers
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const uint32_t chunks = (uint32_t)((n + 63) / 64);
        const uint32_t blocks = std::min<uint32_t>((uint32_t)cus * 2u, (chunks + 3) / 4);
        const hipError_t e = hipMemsetAsync(d_flag, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(k_decode_frames_pipe, dim3(blocks), dim3(256), 0, st, (const uint32_t*)d_bytes, nbytes, d_offsets,
                           (uint32_t)n, sender_override, d_silo_tab, (uint4*)d_out, d_status, d_n_bad, d_flag);
        hipLaunchKernelGGL(k_decode_deferred, grid, dim3(256), 0, st, (const uint32_t*)d_bytes, nbytes, d_offsets,
                           (uint32_t)n, sender_override, d_silo_tab, (uint4*)d_out, d_status, d_n_bad, (const uint32_t*)d_flag);
    } else {
        hipLaunchKernelGGL(k_decode_frames, grid, dim3(256), 0, st, (const uint32_t*)d_bytes, nbytes, d_offsets,
                           (uint32_t)n, sender_override, d_silo_tab, (uint4*)d_out, d_status, d_n_bad);
    }
    return (int)hipGetLastError();
}

}  // namespace orl

namespace orl {

int launch_stamp_frames(const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_offsets, size_t n, const uint32_t* d_route,
                        const uint32_t* d_act, const orl_grain_key* d_act_keys, uint32_t n_act_keys,
                        const orl_grain_key* d_new_act_keys, const GrainTypeEntry* d_gt, const uint8_t* d_gt_blob,
                        const uint32_t* d_silo_words, uint64_t* d_sizes, void* d_temp, size_t temp_bytes, uint8_t* d_out,
                        uint64_t out_cap, uint64_t* d_out_offsets, uint64_t* d_out_total, uint8_t* d_status, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) return (int)hipMemsetAsync(d_out_total, 0, sizeof(uint64_t), st);
    const dim3 grid((uint32_t)((n + 255) / 256));
    const uint32_t* buf = (const uint32_t*)d_bytes;
    uint32_t* out = (uint32_t*)d_out;
    uint32_t* flag = (uint32_t*)(d_sizes + n);  // d_sizes holds n + 1 words: the last one is the deferral flag
    const bool pipe = n >= kPipeMinFrames && nbytes >= 8;
    uint32_t blocks = 0;
    if (pipe) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        blocks = std::min<uint32_t>((uint32_t)cus * 2u, (uint32_t)(((n + 63) / 64 + 3) / 4));
        const hipError_t e = hipMemsetAsync(flag, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return (int)e;
    }
    // pass 1: output sizes
    if (pipe) {
        hipLaunchKernelGGL(k_stamp_pipe<false>, dim3(blocks), dim3(256), 0, st, buf, nbytes, d_offsets, (uint32_t)n, d_route,
                           d_act, d_act_keys, n_act_keys, d_new_act_keys, d_gt, d_gt_blob, d_silo_words, d_sizes,
                           (const uint64_t*)nullptr, out, out_cap, d_status, flag);
        hipLaunchKernelGGL((k_stamp<false, true>), grid, dim3(256), 0, st, buf, nbytes, d_offsets, (uint32_t)n, d_route, d_act,
                           d_act_keys, n_act_keys, d_new_act_keys, d_gt, d_gt_blob, d_silo_words, d_sizes,
                           (const uint64_t*)nullptr, out, out_cap, d_status, (const uint32_t*)flag);
    } else {
        hipLaunchKernelGGL((k_stamp<false, false>), grid, dim3(256), 0, st, buf, nbytes, d_offsets, (uint32_t)n, d_route, d_act,
                           d_act_keys, n_act_keys, d_new_act_keys, d_gt, d_gt_blob, d_silo_words, d_sizes,
                           (const uint64_t*)nullptr, out, out_cap, d_status, (const uint32_t*)flag);
    }
    // output offsets = exclusive scan of the 4-byte-aligned sizes
    size_t tb = temp_bytes;
    hipError_t e = rocprim::exclusive_scan(d_temp, tb, d_sizes, d_out_offsets, (uint64_t)0, n, rocprim::plus<uint64_t>(), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_stamp_total, dim3(1), dim3(1), 0, st, (const uint64_t*)d_sizes, (const uint64_t*)d_out_offsets,
                       (uint32_t)n, d_out_total);
    // pass 2: write
    if (pipe) {
        hipLaunchKernelGGL(k_stamp_pipe<true>, dim3(blocks), dim3(256), 0, st, buf, nbytes, d_offsets, (uint32_t)n, d_route,
                           d_act, d_act_keys, n_act_keys, d_new_act_keys, d_gt, d_gt_blob, d_silo_words, d_sizes,
                           (const uint64_t*)d_out_offsets, out, out_cap, d_status, flag);
        hipLaunchKernelGGL((k_stamp<true, true>), grid, dim3(256), 0, st, buf, nbytes, d_offsets, (uint32_t)n, d_route, d_act,
                           d_act_keys, n_act_keys, d_new_act_keys, d_gt, d_gt_blob, d_silo_words, d_sizes,
                           (const uint64_t*)d_out_offsets, out, out_cap, d_status, (const uint32_t*)flag);
    } else {
        hipLaunchKernelGGL((k_stamp<true, false>), grid, dim3(256), 0, st, buf, nbytes, d_offsets, (uint32_t)n, d_route, d_act,
                           d_act_keys, n_act_keys, d_new_act_keys, d_gt, d_gt_blob, d_silo_words, d_sizes,
                           (const uint64_t*)d_out_offsets, out, out_cap, d_status, (const uint32_t*)flag);
    }
    return (int)hipGetLastError();
}

size_t stamp_scan_temp_bytes(size_t n) {
    size_t tb = 0;
    (void)rocprim::exclusive_scan(nullptr, tb, (const uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, n,
                                  rocprim::plus<uint64_t>(), (hipStream_t)0);
    return tb;
}

}  // namespace orl
