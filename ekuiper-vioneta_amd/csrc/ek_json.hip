// ek_json.hip — columnar JSON ingest on the GPU (north-star item 1).
//
// Replaces, for flat JSON objects with numeric, string and boolean fields, the reference's per-message decode
//   FastJsonConverter.Decode -> decodeWithSchema -> decodeObject   internal/converter/json/converter.go:92-171,246-410
//   extractNumberValue (schema BIGINT -> Int64, FLOAT -> Float64)  converter.go:429-460
//   extractStringValue / extractBooleanFromValue / getBooleanFromValue  converter.go:462-505,600-625
// STRING fields leave as dense u32 dictionary ids (the engine's key column type; see the dictionary section below),
// BOOLEAN fields as int64 0 / 1 that the engine evaluates as Go bools (EK_COL_BOOL).
// A micro-batch of messages (concatenated payload bytes + offsets) is parsed by one thread per message
// straight into the columns of an ek_batch in device memory (one pass, no per-message maps).
//
// Semantics kept from the reference for a schema-typed stream:
//   * a field outside the schema is skipped (checkSchema: not added), null -> nil (validity 0),
//     an absent field -> nil; for duplicate keys the last one wins (obj.Visit + map assignment)
//   * BIGINT: the number must be an integer literal that fits int64 (fastfloat.ParseInt64), else error
//   * FLOAT: the number as float64, correctly rounded (fastfloat.Parse / strconv.ParseFloat)
//   * a string / bool / object / array value for a numeric schema field -> "has wrong type" error
//   * STRING: a JSON string (unescaped as fastjson does); a bool / object / array -> "has wrong type"; a number ->
//     cast.ToStringAlways(float64) on the host converter (EK_JSON_ERR_UNSUPPORTED here)
//   * BOOLEAN: true / false; a number -> != 0 (cast.ToBool, pkg/cast/cast.go:809-837); a string -> strconv.ParseBool;
//     an object / array -> "has wrong type"
//   * any syntax error -> the message fails to decode; the message is dropped and its error reported
//     (DecodeOp forwards the error, node/decode_op.go:146-193)
// Numbers are converted exactly on the Clinger fast path (mantissa <= 2^53, |exp10| <= 22: one IEEE
// multiply/divide by an exact power of ten), else by Eisel-Lemire with a 128-bit power-of-five table,
// whose undecided cases are settled by an exact big-integer midpoint comparison. Not decided on the GPU
// (reported as EK_JSON_ERR_NUMBER, never guessed): subnormal / overflowing results, and mantissas beyond
// 19 significant digits whose truncation straddles a rounding boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ekgpu.h"
#include "ek_errmsg.h"
#include "ek_json_pow5.h"

namespace {

constexpr int kJBlock = 256;

constexpr int kMaxSeg = 8;                     // path segments per column (ABI v14 paths)
constexpr int32_t kStrNumber = 0x20000000;     // slen flag: a number a STRING field received (soff = its f64 bits)
constexpr int32_t kStrFlags = EK_JSON_STR_ESCAPED | kStrNumber;
constexpr uint8_t kErrPending = 0x80;          // first pass: a top-level array payload (decoded by the row-based pass)

struct JSchema {
    int32_t n;
    int32_t type[EK_MAX_COLUMNS];
    int32_t elem[EK_MAX_COLUMNS];                  // EK_COL_LIST: element type
    int32_t nseg[EK_MAX_COLUMNS];                  // path length (1: a top-level field)
    int32_t seg_idx[EK_MAX_COLUMNS][kMaxSeg];      // -1: key segment; >= 0: array element index
    int32_t seg_off[EK_MAX_COLUMNS][kMaxSeg];      // key segment: its bytes name[c][off, off + len)
    int32_t seg_len[EK_MAX_COLUMNS][kMaxSeg];
    uint64_t seg_hash[EK_MAX_COLUMNS][kMaxSeg];    // FNV-1a 64 of the key segment
    uint32_t all;                                  // mask of the schema's columns
    int32_t paths;                                 // some column has nseg > 1
    char name[EK_MAX_COLUMNS][EK_JSON_MAX_NAME];
};

struct JAux {
    unsigned int nulls[EK_MAX_COLUMNS];            // decoded rows with column c nil (0 -> no validity array)
    unsigned int pending;                          // first pass: some message is a top-level array
    unsigned int pad;
    unsigned long long lcnt[EK_MAX_COLUMNS];       // LIST columns: elements reserved
};

struct JOut {
    void* col[EK_MAX_COLUMNS];
    uint8_t* valid[EK_MAX_COLUMNS];
    int64_t* soff[EK_MAX_COLUMNS];   // string columns: the value's first content byte (offset into the payload)
    int32_t* slen[EK_MAX_COLUMNS];   // ... its raw length, | EK_JSON_STR_ESCAPED when it holds a backslash escape;
                                     // LIST columns: the row's element count (col = its first element)
    int64_t* lval[EK_MAX_COLUMNS];   // LIST columns: elements
    uint8_t* lvalid[EK_MAX_COLUMNS];
    uint8_t* err;                    // per message
    uint8_t* rerr;                   // per row (== err when every message is one row)
    const int64_t* rowbase;          // row of message i's first row (nullptr: row i = message i)
    JAux* aux;
};

// strconv.ParseBool over raw string content (cast.ToBool(string, CONVERT_ALL), converter.go:600-625): 1 true, 0 false,
// -1 not a bool literal
__device__ int parse_bool_str(const uint8_t* s, int n) {
    auto is = [&](const char* w) {
        int k = 0;
        for (; w[k]; ++k) if (k >= n || s[k] != (uint8_t)w[k]) return false;
        return k == n;
    };
    if (is("1") || is("t") || is("T") || is("TRUE") || is("true") || is("True")) return 1;
    if (is("0") || is("f") || is("F") || is("FALSE") || is("false") || is("False")) return 0;
    return -1;
}

__device__ __forceinline__ bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

__device__ const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Eisel-Lemire core (Go's strconv eiselLemire64 with its bail-outs reported instead of taken): the
// binary64 bits of w * 10^q from a truncated 128-bit product. *ambiguous: the product could not decide
// the rounding (the true value is then either the candidate or the next double up, since truncation
// only underestimates). Returns false for results outside the normal range.
__device__ bool el_core(uint64_t w, int64_t q, uint64_t* bits, bool* ambiguous) {
    *ambiguous = false;
    const int clz = __clzll((long long)w);
    w <<= clz;
    int64_t exp2 = ((217706 * q) >> 16) + 64 + 1023 - clz;
    const uint64_t hi5 = kPow5Hi[q + 342], lo5 = kPow5Lo[q + 342];
    uint64_t xhi = __umul64hi(w, hi5), xlo = w * hi5;
    if ((xhi & 0x1FF) == 0x1FF && xlo + w < w) {
        const uint64_t yhi = __umul64hi(w, lo5), ylo = w * lo5;
        uint64_t mhi = xhi;
        const uint64_t mlo = xlo + yhi;
        if (mlo < xlo) mhi++;
        if ((mhi & 0x1FF) == 0x1FF && mlo + 1 == 0 && ylo + w < w) *ambiguous = true;
        xhi = mhi;
        xlo = mlo;
    }
    const uint64_t msb = xhi >> 63;
    uint64_t mant = xhi >> (msb + 9);
    exp2 -= (int64_t)(1 ^ msb);
    if (xlo == 0 && (xhi & 0x1FF) == 0 && (mant & 3) == 1) *ambiguous = true;   // half-way at the truncated level
    mant += mant & 1;
    mant >>= 1;
    if ((mant >> 53) > 0) { mant >>= 1; exp2 += 1; }
    if (exp2 <= 0 || exp2 >= 0x7FF) return false;   // subnormal / overflow (ParseFloat range error)
    *bits = ((uint64_t)exp2 << 52) | (mant & 0x000FFFFFFFFFFFFFull);
    return true;
}

// Exact decision for an ambiguous product: compare w * 10^q with the midpoint between the candidate c0
// and the next double up, in big-integer arithmetic (32-bit limbs, values up to ~900 bits).
constexpr int kLimbs = 42;   // 1344 bits: 100 decimal digits (333 bits) times 5^342 (795 bits) plus shifts
struct Big {
    uint32_t d[kLimbs];
};
__device__ void big_set(Big& a, uint64_t v) {
    for (int k = 0; k < kLimbs; ++k) a.d[k] = 0;
    a.d[0] = (uint32_t)v;
    a.d[1] = (uint32_t)(v >> 32);
}
__device__ void big_mul_small(Big& a, uint32_t m) {
    uint64_t carry = 0;
    for (int k = 0; k < kLimbs; ++k) {
        const uint64_t t = (uint64_t)a.d[k] * m + carry;
        a.d[k] = (uint32_t)t;
        carry = t >> 32;
    }
}
__device__ void big_mul_pow5(Big& a, int64_t k) {
    while (k >= 13) { big_mul_small(a, 1220703125u); k -= 13; }   // 5^13 < 2^32
    uint32_t m = 1;
    while (k-- > 0) m *= 5;
    if (m != 1) big_mul_small(a, m);
}
__device__ void big_shl(Big& a, int64_t s) {
    const int w = (int)(s >> 5), b = (int)(s & 31);
    for (int k = kLimbs - 1; k >= 0; --k) {
        const int src = k - w;
        uint32_t v = src >= 0 ? a.d[src] << b : 0u;
        if (b && src - 1 >= 0) v |= a.d[src - 1] >> (32 - b);
        a.d[k] = v;
    }
}
__device__ int big_cmp(const Big& a, const Big& b) {
    for (int k = kLimbs - 1; k >= 0; --k)
        if (a.d[k] != b.d[k]) return a.d[k] < b.d[k] ? -1 : 1;
    return 0;
}
// A (the decimal mantissa) * 10^q vs the midpoint above c0: returns c0 or the next double up
__device__ __noinline__ uint64_t decide_exact_big(Big& A, int64_t q, uint64_t c0) {
    const int64_t e = (int64_t)((c0 >> 52) & 0x7FF);
    const uint64_t m = (c0 & 0x000FFFFFFFFFFFFFull) | (1ull << 52);   // c0 = m * 2^(e - 1075)
    const int64_t E = e - 1076;                                        // midpoint = (2m + 1) * 2^E
    Big B;
    big_set(B, 2 * m + 1);
    // w * 10^q  vs  (2m+1) * 2^E   <=>   A vs B * 2^(E - q), with the power of five on the proper side
    if (q >= 0) big_mul_pow5(A, q); else big_mul_pow5(B, -q);
    const int64_t s = E - q;
    if (s >= 0) big_shl(B, s); else big_shl(A, -s);
    const int c = big_cmp(A, B);
    if (c > 0 || (c == 0 && (m & 1))) return c0 + 1;   // above the midpoint, or a tie to the even neighbour
    return c0;
}
__device__ uint64_t decide_exact(uint64_t w, int64_t q, uint64_t c0) {
    Big A;
    big_set(A, w);
    return decide_exact_big(A, q, c0);
}

// sign of w * 10^q - K * 2^-1075 for q < 0 (K odd: a midpoint between two subnormals): both sides times 2^1075 * 5^-q,
// w * 2^(q + 1075) vs K * 5^-q (at most ~850 bits each)
__device__ int sub_mid_cmp(uint64_t w, int64_t q, uint64_t K) {
    Big A, B;
    big_set(A, w);
    big_set(B, K);
    big_shl(A, q + 1075);
    big_mul_pow5(B, -q);
    return big_cmp(A, B);
}

// A result below 2^-1022 (strconv.ParseFloat returns subnormals without error): m = w * 10^q / 2^-1074 rounded half to
// even, from a double-precision guess corrected by exact midpoint comparisons (the guess is within a few units).
// bits = m is the binary64 encoding (m = 2^52 is the smallest normal). false: not decided (a guess far off).
__device__ __noinline__ bool subnormal_exact(uint64_t w, int64_t q, uint64_t* bits) {
    if (q >= 0) return false;
    const double x = (double)w * pow(10.0, (double)(q + 300));   // q in [-343, -308]: a normal double
    double g = x * ldexp(1e-300, 1074);
    if (!(g >= 0.0) || g > 9007199254740992.0) g = 4503599627370496.0;
    int64_t m = (int64_t)llrint(g);
    for (int it = 0; it < 64; ++it) {
        if (m > 0) {
            const int c = sub_mid_cmp(w, q, 2 * (uint64_t)m - 1);
            if (c < 0 || (c == 0 && (m & 1))) { m--; continue; }
        }
        const int c = sub_mid_cmp(w, q, 2 * (uint64_t)m + 1);
        if (c > 0 || (c == 0 && (m & 1))) { m++; continue; }
        if (m > (int64_t)(1ll << 52)) return false;
        *bits = (uint64_t)m;
        return true;
    }
    return false;
}

// w * 10^q correctly rounded (|w| < 2^64, subnormal results included); false for overflowing results.
__device__ bool dec_to_f64(uint64_t w, int64_t q, bool neg, double* out) {
    if (w == 0 || q < -342) { *out = neg ? -0.0 : 0.0; return true; }   // below 2^-1075 for any 64-bit w
    if (q > 308) return false;
    uint64_t bits;
    bool amb;
    if (!el_core(w, q, &bits, &amb)) {
        // below the normal range (el_core's exponent <= 0; an overflow has q >= 290): decide the subnormal exactly
        if (q > -290 || !subnormal_exact(w, q, &bits)) return false;
        amb = false;
    }
    if (amb) bits = decide_exact(w, q, bits);
    if (((bits >> 52) & 0x7FF) == 0x7FF) return false;
    if (neg) bits |= 1ull << 63;
    *out = __longlong_as_double((long long)bits);
    return true;
}

// Parse a JSON number at p (p < e). Returns the position after it, or nullptr on a syntax error.
struct Num {
    bool neg, is_int, fits_i64, exact, trunc;
    uint64_t mant;       // first <= 19 significant digits
    int64_t exp10;       // value = mant * 10^exp10 (when !trunc)
    int64_t i64;
    double f64;
};

__device__ const uint8_t* parse_number(const uint8_t* p, const uint8_t* e, Num* n) {
    n->neg = false;
    n->is_int = true;
    n->trunc = false;
    n->mant = 0;
    n->exp10 = 0;
    if (p < e && *p == '-') { n->neg = true; ++p; }
    if (p >= e || *p < '0' || *p > '9') return nullptr;
    int nd = 0;            // significant digits kept in mant
    int64_t drop = 0;      // integer digits dropped (beyond 19)
    const uint8_t* ds = p;
    const uint8_t *fs = nullptr, *fe = nullptr;   // fraction digits [fs, fe)
    if (*p == '0') ++p;
    else
        while (p < e && *p >= '0' && *p <= '9') {
            if (nd < 19) { n->mant = n->mant * 10 + (*p - '0'); if (n->mant) nd++; }
            else { drop++; if (*p != '0') n->trunc = true; }
            ++p;
        }
    const int int_digits = (int)(p - ds);
    int64_t frac_exp = 0;
    if (p < e && *p == '.') {
        n->is_int = false;
        ++p;
        if (p >= e || *p < '0' || *p > '9') return nullptr;
        fs = p;
        while (p < e && *p >= '0' && *p <= '9') {
            if (nd < 19) { n->mant = n->mant * 10 + (*p - '0'); frac_exp--; if (n->mant) nd++; }
            else if (*p != '0') n->trunc = true;
            ++p;
        }
        fe = p;
    }
    int64_t ex = 0;
    if (p < e && (*p == 'e' || *p == 'E')) {
        n->is_int = false;
        ++p;
        bool eneg = false;
        if (p < e && (*p == '+' || *p == '-')) { eneg = *p == '-'; ++p; }
        if (p >= e || *p < '0' || *p > '9') return nullptr;
        while (p < e && *p >= '0' && *p <= '9') { if (ex < 100000) ex = ex * 10 + (*p - '0'); ++p; }
        if (eneg) ex = -ex;
    }
    n->exp10 = drop + frac_exp + ex;
    // int64 (fastfloat.ParseInt64): plain integer literal without overflow
    n->fits_i64 = false;
    if (n->is_int && !n->trunc && drop == 0 && int_digits <= 19) {
        const uint64_t lim = n->neg ? (1ull << 63) : ((1ull << 63) - 1);
        if (n->mant <= lim) { n->fits_i64 = true; n->i64 = n->neg ? (int64_t)(0 - n->mant) : (int64_t)n->mant; }
    }
    // float64
    n->exact = true;
    if (!n->trunc && n->mant <= (1ull << 53) && n->exp10 >= -22 && n->exp10 <= 22) {
        double v = (double)n->mant;
        v = n->exp10 < 0 ? __ddiv_rn(v, kPow10[-n->exp10]) : __dmul_rn(v, kPow10[n->exp10]);
        n->f64 = n->neg ? -v : v;
    } else if (!dec_to_f64(n->mant, n->exp10, n->neg, &n->f64)) {
        n->exact = false;   // outside the normal range of binary64
    } else if (n->trunc) {
        // more than 19 significant digits: mant and mant + 1 usually round alike (strconv atof.go); if not,
        // the full digit string (up to 100 significant digits) decides against the midpoint
        double up;
        if (!dec_to_f64(n->mant + 1, n->exp10, n->neg, &up)) n->exact = false;
        else if (up != n->f64 && ((__double_as_longlong(n->f64) >> 52) & 0x7FF) == 0) n->exact = false;   // (subnormal)
        else if (up != n->f64) {
            Big A;
            big_set(A, 0);
            int sig = 0;
            int64_t q = ex;
            const uint8_t* ie = fs ? fs - 1 : (fe ? fe : p);
            if (!fs) ie = ds + int_digits;
            for (const uint8_t* c = ds; c < ie; ++c) {
                if (sig == 0 && *c == '0') continue;
                if (sig >= 100) { q++; continue; }
                big_mul_small(A, 10);
                A.d[0] += *c - '0';   // no carry: the low limb is a multiple of 10 after the multiply
                sig++;
            }
            for (const uint8_t* c = fs; fs && c < fe; ++c) {
                if (sig == 0 && *c == '0') { q--; continue; }
                if (sig >= 100) { if (*c != '0') { n->exact = false; break; } continue; }
                big_mul_small(A, 10);
                A.d[0] += *c - '0';
                sig++;
                q--;
            }
            if (n->exact) {
                // any nonzero integer digit beyond the 100th makes the 100-digit mantissa inexact as well
                int seen = 0;
                for (const uint8_t* c = ds; c < ie; ++c) {
                    if (seen == 0 && *c == '0') continue;
                    if (++seen > 100 && *c != '0') n->exact = false;
                }
            }
            if (n->exact) {
                uint64_t c0 = (uint64_t)__double_as_longlong(n->f64) & ~(1ull << 63);
                const uint64_t b = decide_exact_big(A, q, c0);
                n->f64 = __longlong_as_double((long long)(b | (n->neg ? (1ull << 63) : 0)));
            }
        }
    }
    return p;
}

// skip a JSON string starting at the opening quote; returns the position after the closing quote
__device__ const uint8_t* skip_string(const uint8_t* p, const uint8_t* e) {
    ++p;
    while (p < e) {
        if (*p == '\\') { p += 2; continue; }
        if (*p == '"') return p + 1;
        ++p;
    }
    return nullptr;
}

// skip any JSON value (nested objects/arrays string-aware): one flat scan, in-string state in a flag
__device__ const uint8_t* skip_value(const uint8_t* p, const uint8_t* e) {
    if (p >= e) return nullptr;
    const uint8_t c = *p;
    if (c == '"') return skip_string(p, e);
    if (c == '{' || c == '[') {
        int depth = 0;
        bool in_str = false, esc = false;
        for (; p < e; ++p) {
            const uint8_t x = *p;
            if (in_str) {
                if (esc) esc = false;
                else if (x == '\\') esc = true;
                else if (x == '"') in_str = false;
            } else if (x == '"') {
                in_str = true;
            } else if (x == '{' || x == '[') {
                depth++;
            } else if (x == '}' || x == ']') {
                if (--depth == 0) return p + 1;
            }
        }
        return nullptr;
    }
    if (c == 't') return (e - p >= 4 && p[1] == 'r' && p[2] == 'u' && p[3] == 'e') ? p + 4 : nullptr;
    if (c == 'f') return (e - p >= 5 && p[1] == 'a' && p[2] == 'l' && p[3] == 's' && p[4] == 'e') ? p + 5 : nullptr;
    if (c == 'n') return (e - p >= 4 && p[1] == 'u' && p[2] == 'l' && p[3] == 'l') ? p + 4 : nullptr;
    Num n;
    return parse_number(p, e, &n);
}

__device__ __forceinline__ uint64_t fnv_step(uint64_t h, uint8_t c) { return (h ^ c) * 0x100000001B3ull; }

// One decoded row: the values the row's columns take (ival: int64 / f64 bits / string hash / LIST first element)
struct RowAcc {
    int64_t ival[EK_MAX_COLUMNS];
    int64_t soff[EK_MAX_COLUMNS];
    int32_t slen[EK_MAX_COLUMNS];
    uint32_t seen, isnull;
};

// a JSON string at p (the opening quote): FNV-1a 64 of its raw content, its content range, escape flag; nullptr on a
// syntax error
__device__ __forceinline__ const uint8_t* scan_string(const uint8_t* p, const uint8_t* e, uint64_t* h, const uint8_t** cs,
                                                      int* n_raw, bool* esc) {
    *cs = ++p;
    uint64_t x = 0xCBF29CE484222325ull;
    bool sesc = false;
    while (p < e && *p != '"') {
        if (*p == '\\') {
            sesc = true;
            if (p + 1 >= e) return nullptr;
            x = fnv_step(x, *p);
            ++p;
        }
        x = fnv_step(x, *p);
        ++p;
    }
    if (p >= e) return nullptr;
    *h = x;
    *n_raw = (int)(p - *cs);
    *esc = sesc;
    return p + 1;
}

// One array element of a LIST column (decodeArray, converter.go:173-244, with an Items field of type t): number ->
// extractNumberValue, string -> extractStringValue (a BOOLEAN item through strconv.ParseBool), true / false ->
// extractBooleanFromValue, null -> nil; an object / array item, or a kind the item type does not take, is "array has
// wrong type:%v, expect:%v". Writes *v / *ok; returns the position after it (nullptr: *err set).
__device__ __noinline__ const uint8_t* list_item(int t, const uint8_t* p, const uint8_t* e, int64_t* v, uint8_t* ok, uint8_t* err) {
    const uint8_t c0 = *p;
    *v = 0;
    *ok = 0;
    if (c0 == 'n') {
        p = skip_value(p, e);
        if (!p) *err = EK_JSON_ERR_SYNTAX;
        return p;
    }
    if (c0 == '"') {
        uint64_t h;
        const uint8_t* cs;
        int nr;
        bool esc;
        p = scan_string(p, e, &h, &cs, &nr, &esc);
        if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
        const int b = (t == EK_COL_BOOL && !esc) ? parse_bool_str(cs, nr) : -1;
        if (b < 0) { *err = EK_JSON_ERR_TYPE; return nullptr; }
        *v = b;
        *ok = 1;
        return p;
    }
    if (c0 == 't' || c0 == 'f') {
        p = skip_value(p, e);
        if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
        if (t != EK_COL_BOOL) { *err = EK_JSON_ERR_TYPE; return nullptr; }
        *v = c0 == 't' ? 1 : 0;
        *ok = 1;
        return p;
    }
    if (c0 == '-' || (c0 >= '0' && c0 <= '9')) {
        Num num;
        p = parse_number(p, e, &num);
        if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
        if (t == EK_COL_I64) {
            if (!num.fits_i64) { *err = EK_JSON_ERR_NUMBER; return nullptr; }
            *v = num.i64;
        } else {
            if (!num.exact) { *err = EK_JSON_ERR_NUMBER; return nullptr; }
            *v = t == EK_COL_F64 ? __double_as_longlong(num.f64) : (num.f64 != 0.0 ? 1 : 0);
        }
        *ok = 1;
        return p;
    }
    if (c0 == '{' || c0 == '[') { *err = EK_JSON_ERR_TYPE; return nullptr; }
    *err = EK_JSON_ERR_SYNTAX;
    return nullptr;
}

// The value at p (not null) of leaf column col: the schema type decides the conversion (converter.go:328-400 ->
// extractNumberValue / extractStringValue / extractBooleanFromValue :429-505, getBooleanFromValue :600-625; a LIST
// column decodeArray :173-244). Returns the position after the value (nullptr: *err set).
__device__ const uint8_t* leaf_value(const JSchema& S, int col, const uint8_t* p, const uint8_t* e, const uint8_t* bytes,
                                     RowAcc& R, const JOut& out, uint8_t* err) {
    const uint8_t c0 = *p;
    const int t = S.type[col];
    if (t == EK_COL_LIST) {
        if (c0 != '[') {   // "a has wrong type:number, expect:array"
            *err = (c0 == '-' || (c0 >= '0' && c0 <= '9') || c0 == '"' || c0 == 't' || c0 == 'f' || c0 == '{')
                       ? EK_JSON_ERR_TYPE : EK_JSON_ERR_SYNTAX;
            return nullptr;
        }
        // count the items (one scan), reserve them, then decode them in order
        int64_t cnt = 0;
        const uint8_t* q = p + 1;
        while (q < e && is_ws(*q)) ++q;
        if (q < e && *q == ']') {
            ++q;
        } else {
            for (;;) {
                while (q < e && is_ws(*q)) ++q;
                q = skip_value(q, e);
                if (!q) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
                cnt++;
                while (q < e && is_ws(*q)) ++q;
                if (q < e && *q == ',') { ++q; continue; }
                if (q < e && *q == ']') { ++q; break; }
                *err = EK_JSON_ERR_SYNTAX;
                return nullptr;
            }
        }
        const int64_t base = cnt ? (int64_t)atomicAdd(&out.aux->lcnt[col], (unsigned long long)cnt) : 0;
        const uint8_t* r = p + 1;
        for (int64_t k = 0; k < cnt; ++k) {
            while (r < e && is_ws(*r)) ++r;
            int64_t v;
            uint8_t ok;
            r = list_item(S.elem[col], r, e, &v, &ok, err);
            if (!r) return nullptr;
            out.lval[col][base + k] = v;
            out.lvalid[col][base + k] = ok;
            while (r < e && is_ws(*r)) ++r;
            ++r;   // ',' or ']' (checked by the count scan)
        }
        R.ival[col] = base;
        R.slen[col] = (int32_t)cnt;
        return q;
    }
    if (t == EK_COL_STR || t == EK_COL_BOOL) {
        if (c0 == '"') {
            uint64_t h;
            const uint8_t* cs;
            int n_raw;
            bool sesc;
            p = scan_string(p, e, &h, &cs, &n_raw, &sesc);
            if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
            if (t == EK_COL_STR) {
                R.ival[col] = (int64_t)h;   // FNV-1a 64 of the raw content (= of the string when nothing is escaped)
                R.soff[col] = (int64_t)(cs - bytes);
                R.slen[col] = n_raw | (sesc ? (int32_t)EK_JSON_STR_ESCAPED : 0);
            } else {
                const int b = sesc ? -1 : parse_bool_str(cs, n_raw);
                if (b < 0) { *err = EK_JSON_ERR_TYPE; return nullptr; }   // strconv.ParseBool: invalid syntax
                R.ival[col] = b;
            }
            return p;
        }
        if (c0 == 't' || c0 == 'f') {
            p = skip_value(p, e);
            if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
            if (t == EK_COL_STR) { *err = EK_JSON_ERR_TYPE; return nullptr; }   // "has wrong type:true, expect:string"
            R.ival[col] = c0 == 't' ? 1 : 0;
            return p;
        }
        if (c0 == '-' || (c0 >= '0' && c0 <= '9')) {
            Num num;
            p = parse_number(p, e, &num);
            if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
            if (!num.exact) { *err = EK_JSON_ERR_NUMBER; return nullptr; }
            if (t == EK_COL_STR) {
                // cast.ToStringAlways(float64) (converter.go:446-451): Go's %v of the number, printed by the host
                // dictionary (a miss: the float's bits travel in soff)
                R.ival[col] = 0;
                R.soff[col] = __double_as_longlong(num.f64);
                R.slen[col] = kStrNumber;
            } else {
                R.ival[col] = num.f64 != 0.0 ? 1 : 0;   // cast.ToBool(float64): != 0
            }
            return p;
        }
        *err = (c0 == '{' || c0 == '[') ? EK_JSON_ERR_TYPE : EK_JSON_ERR_SYNTAX;   // object / array: wrong type
        return nullptr;
    }
    if (c0 == '-' || (c0 >= '0' && c0 <= '9')) {
        Num num;
        p = parse_number(p, e, &num);
        if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
        if (t == EK_COL_F64) {
            if (!num.exact) { *err = EK_JSON_ERR_NUMBER; return nullptr; }
            R.ival[col] = __double_as_longlong(num.f64);
        } else {
            if (!num.fits_i64) { *err = EK_JSON_ERR_NUMBER; return nullptr; }
            if (t == EK_COL_U32 && (num.i64 < 0 || num.i64 > 0xFFFFFFFFll)) { *err = EK_JSON_ERR_NUMBER; return nullptr; }
            R.ival[col] = num.i64;
        }
        return p;
    }
    // string / bool / object / array for a numeric schema field (converter.go checkSchema / extract*)
    *err = (c0 == '"' || c0 == 't' || c0 == 'f' || c0 == '{' || c0 == '[') ? EK_JSON_ERR_TYPE : EK_JSON_ERR_SYNTAX;
    return nullptr;
}

// One object (p at its '{') into R: decodeObject (converter.go:246-409) restated over the schema's column paths. Frame
// d is the container at path depth d with the columns whose path runs through it (act); a member whose key (an array
// element whose index) is the next segment of some active column is a leaf of the columns that end there, or the
// container the others descend into; any other member is skipped. Returns the position after the object (nullptr:
// *err set). PATHS = false: every column is a top-level field (depth 0 only).
template <bool PATHS>
__device__ const uint8_t* decode_object(const JSchema& S, const uint8_t* p, const uint8_t* e, const uint8_t* bytes, RowAcc& R,
                                        const JOut& out, uint8_t* err) {
    struct Frame {
        uint32_t act;
        int32_t idx;
        int32_t arr;
    };
    Frame fr[PATHS ? kMaxSeg : 1];
    int d = 0;
    fr[0].act = S.all;
    fr[0].idx = 0;
    fr[0].arr = 0;
    ++p;
    bool open = true;   // the current container has no member yet
    for (;;) {
        while (p < e && is_ws(*p)) ++p;
        if (p >= e) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
        const Frame f = fr[PATHS ? d : 0];
        bool closed = false;
        if (open && *p == (f.arr ? ']' : '}')) {
            ++p;
            closed = true;
        } else {
            uint32_t M = 0;
            if (!f.arr) {
                if (*p != '"') { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
                const uint8_t* ks = ++p;
                uint64_t h = 0xCBF29CE484222325ull;
                bool esc = false;
                while (p < e && *p != '"') {
                    if (*p == '\\') {
                        esc = true;
                        if (++p >= e) break;
                    }
                    h = fnv_step(h, *p);
                    ++p;
                }
                if (p >= e) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
                const int klen = (int)(p - ks);
                ++p;
                if (!esc) {
                    for (uint32_t a = f.act; a; a &= a - 1) {
                        const int c = __ffs(a) - 1;
                        if (S.seg_idx[c][PATHS ? d : 0] >= 0 || S.seg_hash[c][PATHS ? d : 0] != h ||
                            S.seg_len[c][PATHS ? d : 0] != klen)
                            continue;
                        const char* nm = S.name[c] + S.seg_off[c][PATHS ? d : 0];
                        bool eq = true;
                        for (int k = 0; k < klen; ++k) eq &= (uint8_t)nm[k] == ks[k];
                        if (eq) M |= 1u << c;
                    }
                }
                while (p < e && is_ws(*p)) ++p;
                if (p >= e || *p != ':') { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
                ++p;
                while (p < e && is_ws(*p)) ++p;
                if (p >= e) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
            } else {
                const int j = f.idx;
                fr[PATHS ? d : 0].idx = j + 1;
                for (uint32_t a = f.act; a; a &= a - 1) {
                    const int c = __ffs(a) - 1;
                    if (S.seg_idx[c][PATHS ? d : 0] == j) M |= 1u << c;
                }
            }
            const uint8_t c0 = *p;
            if (!M) {
                p = skip_value(p, e);
                if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
            } else {
                uint32_t L = 0, I = 0;
                for (uint32_t a = M; a; a &= a - 1) {
                    const int c = __ffs(a) - 1;
                    if (S.nseg[c] == d + 1) L |= 1u << c;
                    else I |= 1u << c;
                }
                if (c0 == 'n') {
                    // nil: the leaves are nil, and so is every leaf below a nil container (m[key] = nil)
                    p = skip_value(p, e);
                    if (!p) { *err = EK_JSON_ERR_SYNTAX; return nullptr; }
                    R.seen |= M;
                    R.isnull |= M;
                } else if (PATHS && I) {
                    // the path continues: the value must be the container kind the next segments name
                    // ("a has wrong type:number, expect:struct"; a scalar leaf column on the same key gets a container)
                    uint32_t want_arr = 0;
                    for (uint32_t a = I; a; a &= a - 1) {
                        const int c = __ffs(a) - 1;
                        if (S.seg_idx[c][d + 1] >= 0) want_arr |= 1u << c;
                    }
                    const bool ok = (c0 == '{' && !want_arr) || (c0 == '[' && want_arr == I);
                    if (!ok) {
                        *err = (c0 == '{' || c0 == '[' || c0 == '"' || c0 == 't' || c0 == 'f' || c0 == '-' ||
                                (c0 >= '0' && c0 <= '9')) ? EK_JSON_ERR_TYPE : EK_JSON_ERR_SYNTAX;
                        return nullptr;
                    }
                    if (L) { *err = EK_JSON_ERR_UNSUPPORTED; return nullptr; }   // a column ends where another descends
                    // a repeated key replaces the whole subtree (Go map assignment): its leaves start unseen again
                    R.seen &= ~I;
                    R.isnull &= ~I;
                    ++d;
                    fr[d].act = I;
                    fr[d].idx = 0;
                    fr[d].arr = c0 == '[';
                    ++p;
                    open = true;
                    continue;
                } else {
                    const uint8_t* q = p;
                    for (uint32_t a = L; a; a &= a - 1) {   // (two columns may name one field)
                        const int c = __ffs(a) - 1;
                        q = leaf_value(S, c, p, e, bytes, R, out, err);
                        if (!q) return nullptr;
                    }
                    p = q;
                    R.seen |= L;
                    R.isnull &= ~L;
                }
            }
        }
        // separators and closing brackets back up the frames
        for (;;) {
            if (closed) {
                if (d == 0) return p;
                --d;
            }
            while (p < e && is_ws(*p)) ++p;
            const uint8_t cl = fr[PATHS ? d : 0].arr ? ']' : '}';
            if (p < e && *p == ',') { ++p; open = false; break; }
            if (p < e && *p == cl) { ++p; closed = true; continue; }
            *err = EK_JSON_ERR_SYNTAX;
            return nullptr;
        }
    }
}

__device__ __forceinline__ void emit_row(const JSchema& S, const JOut& out, int64_t r, const RowAcc& R, bool good) {
    for (int c = 0; c < S.n; ++c) {
        const bool ok = good && ((R.seen >> c) & 1u) && !((R.isnull >> c) & 1u);
        if (good && !ok) atomicAdd(&out.aux->nulls[c], 1u);
        if (out.valid[c]) out.valid[c][r] = ok ? 1 : 0;
        const int64_t v = ok ? R.ival[c] : 0;
        if (S.type[c] == EK_COL_U32) ((uint32_t*)out.col[c])[r] = (uint32_t)v;
        else ((int64_t*)out.col[c])[r] = v;
        if (S.type[c] == EK_COL_STR) {
            out.soff[c][r] = ok ? R.soff[c] : 0;
            out.slen[c][r] = ok ? R.slen[c] : 0;
        } else if (S.type[c] == EK_COL_LIST) {
            out.slen[c][r] = ok ? R.slen[c] : 0;
        }
    }
}

// One thread per message: an object is one row; a top-level array of objects (decodeWithSchema's []map case,
// converter.go:141-158) is one row per element, at rows [rowbase[i], rowbase[i + 1]) (first pass, rowbase = nullptr:
// the message is marked pending and decoded by the row-based pass). Errors fail the whole message.
// The block's messages are contiguous in the payload: when they fit kJStage bytes they are first copied into LDS with
// 16-byte loads (consecutive lanes on consecutive chunks) and every thread parses its message from there — a thread's
// byte loads straight from HBM touch a different line per lane (one line per lane per byte step), the LDS copy reads
// each line once. String offsets stay payload offsets (src maps payload offset g to the LDS copy of byte g).
constexpr int kJStage = 16384;
template <bool PATHS>
__global__ __launch_bounds__(kJBlock) void k_json_decode(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off,
                                                         int64_t n, const JSchema* __restrict__ sch, JOut out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_msg[kJStage];
    const int64_t i = (int64_t)blockIdx.x * kJBlock + threadIdx.x;
    const uint8_t* src = bytes;
    {
        const int64_t b0 = (int64_t)blockIdx.x * kJBlock, b1 = b0 + kJBlock < n ? b0 + kJBlock : n;
        const uintptr_t a_lo = (uintptr_t)(bytes + off[b0]), a_hi = (uintptr_t)(bytes + off[b1]);
        const uintptr_t base = a_lo & ~(uintptr_t)15;
        if (a_hi > a_lo && a_hi - base <= (uintptr_t)kJStage) {   // uniform over the block
            const uintptr_t f_lo = (a_lo + 15) & ~(uintptr_t)15, f_hi = a_hi & ~(uintptr_t)15;   // whole chunks inside
            uintptr_t h1 = a_hi, t0 = a_hi;
            if (f_lo < f_hi) {
                for (uintptr_t a = f_lo + 16 * (uintptr_t)threadIdx.x; a < f_hi; a += 16 * (uintptr_t)kJBlock)
                    *(uint4*)(s_msg + (a - base)) = *(const uint4*)a;
                h1 = f_lo;
                t0 = f_hi;
            }
            for (uintptr_t a = a_lo + threadIdx.x; a < h1; a += kJBlock) s_msg[a - base] = *(const uint8_t*)a;
            for (uintptr_t a = t0 + threadIdx.x; a < a_hi; a += kJBlock) s_msg[a - base] = *(const uint8_t*)a;
            __syncthreads();
            src = (const uint8_t*)((uintptr_t)(const uint8_t*)s_msg - (base - (uintptr_t)bytes));
        }
    }
    if (i >= n) return;
    const JSchema& S = *sch;
    const uint8_t* p = src + off[i];
    const uint8_t* e = src + off[i + 1];
    RowAcc R;
    R.seen = 0;
    R.isnull = 0;
    uint8_t err = EK_JSON_OK;
    const int64_t r0 = out.rowbase ? out.rowbase[i] : i;
    const int64_t nr = out.rowbase ? out.rowbase[i + 1] - r0 : 1;
    int64_t done = 0;
    while (p < e && is_ws(*p)) ++p;
    if (p < e && *p == '{') {
        p = decode_object<PATHS>(S, p, e, src, R, out, &err);
        if (p) {
            emit_row(S, out, r0, R, true);
            done = 1;
        }
    } else if (p < e && *p == '[') {
        if (!out.rowbase) {
            err = kErrPending;
            atomicOr(&out.aux->pending, 1u);
        } else {
            ++p;
            while (p < e && is_ws(*p)) ++p;
            if (p < e && *p == ']') {
                ++p;
            } else {
                for (;;) {
                    while (p < e && is_ws(*p)) ++p;
                    // every element must be an object ("value doesn't contain object", converter.go:147-150)
                    if (p >= e || *p != '{' || done >= nr) { err = (p < e && *p != '{') ? EK_JSON_ERR_TYPE : EK_JSON_ERR_SYNTAX; break; }
                    R.seen = 0;
                    R.isnull = 0;
                    p = decode_object<PATHS>(S, p, e, src, R, out, &err);
                    if (!p) break;
                    emit_row(S, out, r0 + done, R, true);
                    done++;
                    while (p < e && is_ws(*p)) ++p;
                    if (p < e && *p == ',') { ++p; continue; }
                    if (p < e && *p == ']') { ++p; break; }
                    err = EK_JSON_ERR_SYNTAX;
                    break;
                }
            }
        }
    } else {
        err = EK_JSON_ERR_SYNTAX;   // not an object / array payload (decodeWithSchema's "only map ... is supported")
    }
    if (err == EK_JSON_OK) {
        while (p < e && is_ws(*p)) ++p;
        if (p != e) err = EK_JSON_ERR_SYNTAX;   // trailing bytes after the value
        else if (done != nr) err = EK_JSON_ERR_SYNTAX;   // (the row count scan disagreed)
    }
    out.err[i] = err;
    if (out.rerr != out.err)
        for (int64_t k = 0; k < nr; ++k) out.rerr[r0 + k] = err;
    if (err != EK_JSON_OK) {
        // a failed message leaves no row: its rows are dropped by the compaction (valid bytes zeroed for determinism)
        R.seen = 0;
        for (int64_t k = (out.rowbase ? 0 : done); k < nr; ++k) emit_row(S, out, r0 + k, R, false);
    }
}

// rows of every message (row-based pass): 1 for an object, the element count of a top-level array
__global__ __launch_bounds__(kJBlock) void k_json_rows(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ off,
                                                       int64_t n, int64_t* __restrict__ rows) {
    const int64_t i = (int64_t)blockIdx.x * kJBlock + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = bytes + off[i];
    const uint8_t* e = bytes + off[i + 1];
    while (p < e && is_ws(*p)) ++p;
    int64_t c = 1;
    if (p < e && *p == '[') {
        c = 0;
        ++p;
        while (p < e && is_ws(*p)) ++p;
        if (p < e && *p != ']') {
            for (;;) {
                while (p < e && is_ws(*p)) ++p;
                p = skip_value(p, e);
                if (!p) break;
                c++;
                while (p < e && is_ws(*p)) ++p;
                if (p < e && *p == ',') { ++p; continue; }
                break;
            }
        }
    }
    rows[i] = c;
}

// stable compaction of the messages that decoded (same scheme as the range-mode trigger lists)
constexpr int kTile = 4096;
__global__ __launch_bounds__(kJBlock) void k_ok_count(const uint8_t* __restrict__ err, int64_t n, int64_t* cnt) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    int64_t c = 0;
    for (int k = threadIdx.x; k < kTile; k += kJBlock) { const int64_t i = base + k; if (i < n && err[i] == 0) c++; }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ int64_t s[kJBlock / 64];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ __launch_bounds__(1024) void k_scan_cnt(int64_t* cnt, int nb) {
    __shared__ int64_t part[1024];
    const int per = (nb + 1023) / 1024;
    const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    int64_t s = 0;
    for (int k = b0; k < b1; ++k) s += cnt[k];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t run = 0;
        for (int t = 0; t < 1024; ++t) { int64_t x = part[t]; part[t] = run; run += x; }
        cnt[nb] = run;
    }
    __syncthreads();
    int64_t run = part[threadIdx.x];
    for (int k = b0; k < b1; ++k) { int64_t x = cnt[k]; cnt[k] = run; run += x; }
}
// move the decoded rows down to their compacted positions (row k -> dest <= k, processed in order per block)
__global__ __launch_bounds__(kJBlock) void k_ok_pos(const uint8_t* __restrict__ err, int64_t n, const int64_t* cnt,
                                                    int64_t* __restrict__ pos) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    __shared__ uint32_t wsum[kJBlock / 64];
    int64_t run = cnt[blockIdx.x];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k0 = 0; k0 < kTile; k0 += kJBlock) {
        const int64_t i = base + k0 + threadIdx.x;
        const bool f = i < n && err[i] == 0;
        const unsigned long long m = __ballot(f);
        if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t wb = 0, tot = 0;
        for (int w = 0; w < kJBlock / 64; ++w) { if (w < wv) wb += wsum[w]; tot += wsum[w]; }
        if (i < n) pos[i] = f ? run + wb + __popcll(m & ((1ull << lane) - 1ull)) : -1;
        run += tot;
        __syncthreads();
    }
}
// exclusive scan of the rows per message -> rowbase[0..n] (per 4096-message tile: sum, tile offsets, block scan)
__global__ __launch_bounds__(kJBlock) void k_rows_tile_sum(const int64_t* __restrict__ rows, int64_t n, int64_t* tsum) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    int64_t c = 0;
    for (int k = threadIdx.x; k < kTile; k += kJBlock) { const int64_t i = base + k; if (i < n) c += rows[i]; }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ int64_t s[kJBlock / 64];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tsum[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ __launch_bounds__(kJBlock) void k_rows_tile_scan(const int64_t* __restrict__ rows, int64_t n,
                                                            const int64_t* __restrict__ tsum, int nb,
                                                            int64_t* __restrict__ rowbase) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    __shared__ int64_t wsum[kJBlock / 64];
    int64_t run = tsum[blockIdx.x];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k0 = 0; k0 < kTile; k0 += kJBlock) {
        const int64_t i = base + k0 + threadIdx.x;
        const int64_t v = i < n ? rows[i] : 0;
        int64_t x = v;
        for (int o = 1; o < 64; o <<= 1) { const int64_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        int64_t wb = 0, tot = 0;
        for (int w = 0; w < kJBlock / 64; ++w) { if (w < wv) wb += wsum[w]; tot += wsum[w]; }
        if (i < n) rowbase[i] = run + wb + x - v;
        run += tot;
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) rowbase[n] = tsum[nb];
}
__global__ void k_compact_col(const int64_t* __restrict__ pos, int64_t n, const void* __restrict__ src, void* __restrict__ dst,
                              int es) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t d = pos[i];
        if (d < 0) continue;
        if (es == 8) ((int64_t*)dst)[d] = ((const int64_t*)src)[i];
        else if (es == 4) ((uint32_t*)dst)[d] = ((const uint32_t*)src)[i];
        else ((uint8_t*)dst)[d] = ((const uint8_t*)src)[i];
    }
}

// ---------------------------------------------------------------- STRING columns: the per-column dictionary
// Each STRING column of a decoded batch leaves the decoder as dense u32 ids (first-seen order over the decoder's life),
// the engine's key column type. The device holds an open-addressing table FNV-1a 64 hash -> id (Fibonacci-hashed slot,
// linear probing, load <= 1/2); a row whose hash is in the table takes its id there. The rest — strings never seen
// and strings holding a backslash escape (their device hash covers the escaped form) — are the misses: the host
// reads their bytes, unescapes them (valyala/fastjson v1.6.4 unescapeStringBestEffort, go.mod:82), enters new
// strings in its dictionary and scatters the ids. In steady state (a bounded key set, e.g. deviceId) every row hits
// and the resolution is one kernel plus a 8-byte readback.
struct MissRec {
    int64_t row, off;
    int32_t len, pad;
};
__host__ __device__ __forceinline__ uint64_t str_key(uint64_t h) { return h ? h : 1; }   // 0 marks an empty slot
__host__ __device__ __forceinline__ uint64_t str_slot(uint64_t h, int bits) { return (h * 0x9E3779B97F4A7C15ull) >> (64 - bits); }

__global__ __launch_bounds__(256) void k_str_lookup(const int64_t* __restrict__ hash, const int64_t* __restrict__ soff,
                                                    const int32_t* __restrict__ slen, const uint8_t* __restrict__ valid,
                                                    int64_t n, const uint64_t* __restrict__ tkey,
                                                    const uint32_t* __restrict__ tval, const uint32_t* __restrict__ tlen,
                                                    int bits, uint32_t* __restrict__ id,
                                                    MissRec* __restrict__ miss, unsigned long long* __restrict__ n_miss) {
    const uint64_t mask = bits ? (1ull << bits) - 1ull : 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t v = 0;
        if (valid[i]) {
            const int32_t L = slen[i];
            bool found = false;
            if (!(L & kStrFlags) && bits) {
                const uint64_t h = str_key((uint64_t)hash[i]);
                for (uint64_t k = str_slot(h, bits);; k = (k + 1) & mask) {
                    const uint64_t t = tkey[k];
                    // a hit needs the hash AND the length: a colliding string of another length is a miss, and the
                    // host's resolve (which holds the strings) reports the collision instead of merging the two groups
                    if (t == h && tlen[k] == (uint32_t)L) { v = tval[k]; found = true; break; }
                    if (t == 0) break;
                }
            }
            if (!found) {
                const unsigned long long m = atomicAdd(n_miss, 1ull);
                MissRec r;
                r.row = i;
                r.off = soff[i];
                r.len = L;
                r.pad = 0;
                miss[m] = r;
            }
        }
        id[i] = v;
    }
}
// the misses' bytes (device payloads): record k's string -> dst[dpos[k], dpos[k] + len)
__global__ void k_str_gather(const uint8_t* __restrict__ bytes, const MissRec* __restrict__ miss, const int64_t* __restrict__ dpos,
                             int64_t nm, uint8_t* __restrict__ dst) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nm; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = miss[k].off, d = dpos[k];
        if (miss[k].len & kStrNumber) continue;   // (a number: no payload bytes)
        const int32_t L = miss[k].len & ~kStrFlags;
        for (int32_t j = 0; j < L; ++j) dst[d + j] = bytes[o + j];
    }
}
__global__ void k_str_scatter(const int64_t* __restrict__ rows, const uint32_t* __restrict__ ids, int64_t nm, uint32_t* __restrict__ id) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nm; k += (int64_t)gridDim.x * blockDim.x) id[rows[k]] = ids[k];
}

// fastjson unescapeStringBestEffort (valyala/fastjson v1.6.4 parser.go): \" \\ \/ \b \f \n \r \t, \uXXXX (a surrogate
// pair as one rune, an unpaired or invalid pair as U+FFFD via utf16.DecodeRune), anything else left as is
void utf8_put(std::string& o, uint32_t r) {
    if (r < 0x80) o += (char)r;
    else if (r < 0x800) { o += (char)(0xC0 | (r >> 6)); o += (char)(0x80 | (r & 0x3F)); }
    else if (r < 0x10000) { o += (char)(0xE0 | (r >> 12)); o += (char)(0x80 | ((r >> 6) & 0x3F)); o += (char)(0x80 | (r & 0x3F)); }
    else {
        o += (char)(0xF0 | (r >> 18)); o += (char)(0x80 | ((r >> 12) & 0x3F));
        o += (char)(0x80 | ((r >> 6) & 0x3F)); o += (char)(0x80 | (r & 0x3F));
    }
}
int hex4(const uint8_t* s) {
    int v = 0;
    for (int k = 0; k < 4; ++k) {
        const int c = s[k];
        const int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
        if (d < 0) return -1;
        v = v * 16 + d;
    }
    return v;
}
std::string json_unescape(const uint8_t* s, int64_t n) {
    std::string o;
    o.reserve((size_t)n);
    int64_t i = 0;
    while (i < n) {
        if (s[i] != '\\' || i + 1 >= n) { o += (char)s[i++]; continue; }
        const uint8_t c = s[i + 1];
        switch (c) {
        case '"': o += '"'; i += 2; break;
        case '\\': o += '\\'; i += 2; break;
        case '/': o += '/'; i += 2; break;
        case 'b': o += '\b'; i += 2; break;
        case 'f': o += '\f'; i += 2; break;
        case 'n': o += '\n'; i += 2; break;
        case 'r': o += '\r'; i += 2; break;
        case 't': o += '\t'; i += 2; break;
        case 'u': {
            const int x = i + 6 <= n ? hex4(s + i + 2) : -1;
            if (x < 0) { o += "\\u"; i += 2; break; }
            if (x < 0xD800 || x >= 0xE000) { utf8_put(o, (uint32_t)x); i += 6; break; }
            const int y = (i + 12 <= n && s[i + 6] == '\\' && s[i + 7] == 'u') ? hex4(s + i + 8) : -1;
            if (y < 0) { o += "\\u"; i += 2; break; }
            uint32_t r = 0xFFFD;   // utf16.DecodeRune: a high then a low surrogate, else U+FFFD
            if (x < 0xDC00 && y >= 0xDC00 && y < 0xE000) r = 0x10000 + (((uint32_t)x - 0xD800) << 10) + ((uint32_t)y - 0xDC00);
            utf8_put(o, r);
            i += 12;
            break;
        }
        default: o += '\\'; o += (char)c; i += 2; break;   // unknown escape: kept
        }
    }
    return o;
}
uint64_t fnv1a64(const std::string& s) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (unsigned char c : s) h = (h ^ c) * 0x100000001B3ull;
    return h;
}

struct StrDict {
    std::unordered_map<std::string, uint32_t> ids;
    std::unordered_map<uint64_t, uint32_t> by_key;   // str_key(hash) -> id (collision check)
    std::vector<std::string> values;
    std::vector<uint64_t> hkey;                      // host mirror of the device table
    std::vector<uint32_t> hval;
    std::vector<uint32_t> hlen;                      // the string's byte length: a hash hit must match it too
    int bits = 0;
    bool dirty = false;
    void put(uint64_t key, uint32_t id) {
        const uint64_t mask = (1ull << bits) - 1ull;
        for (uint64_t k = str_slot(key, bits);; k = (k + 1) & mask)
            if (hkey[k] == 0) { hkey[k] = key; hval[k] = id; hlen[k] = (uint32_t)values[id].size(); return; }
    }
    void insert(uint64_t key, uint32_t id) {
        if (bits == 0 || (by_key.size() + 1) * 2 > ((size_t)1 << bits)) {   // grow: load <= 1/2
            bits = std::max(bits + 1, 10);
            while (((size_t)1 << bits) < (by_key.size() + 1) * 2) ++bits;
            hkey.assign((size_t)1 << bits, 0);
            hval.assign((size_t)1 << bits, 0);
            hlen.assign((size_t)1 << bits, 0);
            for (const auto& kv : by_key) put(kv.first, kv.second);
        }
        put(key, id);
        by_key.emplace(key, id);
        dirty = true;
    }
};

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct JsonDecoder {
    int dev = 0;
    JSchema sch{};
    JSchema* d_sch = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    Buf in_bytes, in_off, raw_col[EK_MAX_COLUMNS], raw_valid[EK_MAX_COLUMNS], out_col[EK_MAX_COLUMNS],
        out_valid[EK_MAX_COLUMNS], msg_err, row_err, pos, cnt, aux, rowbase;
    Buf lval[EK_MAX_COLUMNS], lvalid[EK_MAX_COLUMNS];   // LIST columns: the elements (ek_json_list)
    const int64_t* list_start[EK_MAX_COLUMNS] = {};
    const int32_t* list_len[EK_MAX_COLUMNS] = {};
    std::vector<int64_t> h_rows_of;                    // rows per message of the last decode (ek_json_rows)
    Buf raw_soff[EK_MAX_COLUMNS], raw_slen[EK_MAX_COLUMNS], out_soff[EK_MAX_COLUMNS], out_slen[EK_MAX_COLUMNS];
    const int64_t* str_off[EK_MAX_COLUMNS] = {};   // the last decode's string references (ek_json_strings)
    const int32_t* str_len[EK_MAX_COLUMNS] = {};
    StrDict dict[EK_MAX_COLUMNS];
    Buf id_col[EK_MAX_COLUMNS], tkey[EK_MAX_COLUMNS], tval[EK_MAX_COLUMNS], tlen[EK_MAX_COLUMNS], miss, n_miss, gat_pos, gat_bytes, fix_rows, fix_ids;
    std::vector<uint8_t> h_err;
    int64_t last_n = 0, last_ok = 0;
    ek_json_stats st{};

    int fail(int code, const char* fmt, ...) {
        char b[256];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(b, sizeof b, fmt, ap);
        va_end(ap);
        err = b;
        return code;
    }
    int ensure(Buf& b, size_t bytes) {
        if (b.p && b.bytes >= bytes) return 0;
        if (b.p) { hipStreamSynchronize(stream); hipFree(b.p); b.p = nullptr; }
        const size_t nb = std::max<size_t>(bytes, 256);
        if (hipMalloc(&b.p, nb) != hipSuccess) return fail(EK_ERR_NOMEM, "hipMalloc(%zu) failed", nb);
        b.bytes = nb;
        return 0;
    }
    ~JsonDecoder() {
        if (stream) hipStreamSynchronize(stream);
        for (Buf* b : {&in_bytes, &in_off, &msg_err, &row_err, &pos, &cnt, &aux, &rowbase, &miss, &n_miss, &gat_pos, &gat_bytes,
                       &fix_rows, &fix_ids})
            if (b->p) hipFree(b->p);
        for (int c = 0; c < EK_MAX_COLUMNS; ++c)
            for (Buf* b : {&raw_col[c], &raw_valid[c], &out_col[c], &out_valid[c], &raw_soff[c], &raw_slen[c], &out_soff[c],
                           &out_slen[c], &id_col[c], &tkey[c], &tval[c], &tlen[c], &lval[c], &lvalid[c]})
                if (b->p) hipFree(b->p);
        if (d_sch) hipFree(d_sch);
        if (stream) hipStreamDestroy(stream);
    }

    // a column name -> path segments (ABI v14 paths: "a.b", "a[0]", "a[0][0].c"); without paths the name is one key
    int compile_path(int c, const char* nm, size_t L, bool paths) {
        int ns = 0;
        auto key = [&](size_t off, size_t len) {
            if (len == 0 || ns >= kMaxSeg) return false;
            uint64_t h = 0xCBF29CE484222325ull;
            for (size_t k = 0; k < len; ++k) h = (h ^ (uint8_t)nm[off + k]) * 0x100000001B3ull;
            sch.seg_idx[c][ns] = -1;
            sch.seg_off[c][ns] = (int32_t)off;
            sch.seg_len[c][ns] = (int32_t)len;
            sch.seg_hash[c][ns] = h;
            ns++;
            return true;
        };
        if (!paths) {
            key(0, L);
        } else {
            size_t k = 0;
            while (k < L) {
                size_t ke = k;
                while (ke < L && nm[ke] != '.' && nm[ke] != '[') ++ke;
                if (ke > k) {
                    if (!key(k, ke - k)) return fail(EK_ERR_INVALID, "bad path \"%s\"", nm);
                } else if (ns == 0 || nm[k] != '[') {
                    return fail(EK_ERR_INVALID, "bad path \"%s\" (a path starts with a field name)", nm);
                }
                k = ke;
                while (k < L && nm[k] == '[') {
                    size_t q = k + 1;
                    int64_t idx = 0;
                    while (q < L && nm[q] >= '0' && nm[q] <= '9' && idx < (1ll << 30)) idx = idx * 10 + (nm[q++] - '0');
                    if (q == k + 1 || q >= L || nm[q] != ']' || ns >= kMaxSeg)
                        return fail(EK_ERR_INVALID, "bad path \"%s\" (array index)", nm);
                    sch.seg_idx[c][ns] = (int32_t)idx;
                    sch.seg_off[c][ns] = 0;
                    sch.seg_len[c][ns] = 0;
                    sch.seg_hash[c][ns] = 0;
                    ns++;
                    k = q + 1;
                }
                if (k < L) {
                    if (nm[k] != '.' || k + 1 >= L) return fail(EK_ERR_INVALID, "bad path \"%s\"", nm);
                    ++k;
                }
            }
        }
        if (ns == 0) return fail(EK_ERR_INVALID, "bad field name %d", c);
        sch.nseg[c] = ns;
        if (ns > 1) sch.paths = 1;
        return 0;
    }

    int init(const ek_json_schema* s, int device) {
        if (!s || s->n_fields <= 0 || s->n_fields > EK_MAX_COLUMNS) return fail(EK_ERR_INVALID, "bad schema field count");
        sch.n = s->n_fields;
        sch.all = sch.n >= 32 ? 0xFFFFFFFFu : (1u << sch.n) - 1u;
        for (int c = 0; c < sch.n; ++c) {
            const int t = s->column_type[c];
            if (t != EK_COL_I64 && t != EK_COL_F64 && t != EK_COL_U32 && t != EK_COL_STR && t != EK_COL_BOOL && t != EK_COL_LIST)
                return fail(EK_ERR_INVALID, "bad column type");
            sch.type[c] = t;
            if (t == EK_COL_LIST) {
                const int et = s->elem_type[c];
                if (et != EK_COL_I64 && et != EK_COL_F64 && et != EK_COL_BOOL)
                    return fail(EK_ERR_INVALID, "LIST column %d: element type must be BIGINT, FLOAT or BOOLEAN", c);
                sch.elem[c] = et;
            }
            const size_t L = strnlen(s->names[c], EK_JSON_MAX_NAME);
            if (L == 0 || L >= EK_JSON_MAX_NAME) return fail(EK_ERR_INVALID, "bad field name %d", c);
            memcpy(sch.name[c], s->names[c], L);
            if (int rc = compile_path(c, sch.name[c], L, s->paths != 0)) return rc;
        }
        if (hipSetDevice(device) != hipSuccess) return fail(EK_ERR_DEVICE, "hipSetDevice(%d) failed", device);
        dev = device;
        if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return fail(EK_ERR_DEVICE, "stream");
        if (hipMalloc((void**)&d_sch, sizeof(JSchema)) != hipSuccess) return fail(EK_ERR_NOMEM, "schema alloc");
        if (hipMemcpy(d_sch, &sch, sizeof(JSchema), hipMemcpyHostToDevice) != hipSuccess) return fail(EK_ERR_DEVICE, "schema copy");
        return 0;
    }

    int launch_decode(const uint8_t* d_bytes, const int64_t* d_off, int64_t n, const JOut& jo) {
        const dim3 g((unsigned)((n + kJBlock - 1) / kJBlock));
        if (sch.paths) hipLaunchKernelGGL(k_json_decode<true>, g, dim3(kJBlock), 0, stream, d_bytes, d_off, n, d_sch, jo);
        else hipLaunchKernelGGL(k_json_decode<false>, g, dim3(kJBlock), 0, stream, d_bytes, d_off, n, d_sch, jo);
        return 0;
    }
    // the per-row output arrays for `rows` rows (LIST elements: at most one per two payload bytes, plus one per row)
    int row_buffers(int64_t rows, int64_t n_bytes, JOut& jo) {
        const int64_t rr = std::max<int64_t>(rows, 1);
        for (int c = 0; c < sch.n; ++c) {
            const size_t es = sch.type[c] == EK_COL_U32 ? 4 : 8;
            if (int rc = ensure(raw_col[c], (size_t)rr * es)) return rc;
            if (int rc = ensure(raw_valid[c], (size_t)rr)) return rc;
            jo.col[c] = raw_col[c].p;
            jo.valid[c] = (uint8_t*)raw_valid[c].p;
            str_off[c] = nullptr;
            str_len[c] = nullptr;
            list_start[c] = nullptr;
            list_len[c] = nullptr;
            if (sch.type[c] == EK_COL_STR) {
                if (int rc = ensure(raw_soff[c], (size_t)rr * 8)) return rc;
                jo.soff[c] = (int64_t*)raw_soff[c].p;
            }
            if (sch.type[c] == EK_COL_STR || sch.type[c] == EK_COL_LIST) {
                if (int rc = ensure(raw_slen[c], (size_t)rr * 4)) return rc;
                jo.slen[c] = (int32_t*)raw_slen[c].p;
            }
            if (sch.type[c] == EK_COL_LIST) {
                const size_t cap = (size_t)(n_bytes / 2 + rr + 1);
                if (int rc = ensure(lval[c], cap * 8)) return rc;
                if (int rc = ensure(lvalid[c], cap)) return rc;
                jo.lval[c] = (int64_t*)lval[c].p;
                jo.lvalid[c] = (uint8_t*)lvalid[c].p;
            }
        }
        return 0;
    }

    int decode(const char* bytes, int64_t n_bytes, const int64_t* offsets, int64_t n, int32_t memory, ek_batch* out) {
        if (!out || n < 0 || n_bytes < 0 || (n > 0 && (!bytes || !offsets))) return fail(EK_ERR_INVALID, "bad arguments");
        memset(out, 0, sizeof *out);
        out->memory = EK_MEM_DEVICE;
        last_n = n;
        last_ok = 0;
        h_rows_of.clear();
        if (n == 0) return 0;
        const uint8_t* d_bytes = (const uint8_t*)bytes;
        const int64_t* d_off = offsets;
        if (memory == EK_MEM_HOST) {
            if (offsets[0] < 0 || offsets[n] > n_bytes) return fail(EK_ERR_INVALID, "offsets outside the payload");
            if (int rc = ensure(in_bytes, (size_t)n_bytes + 1)) return rc;
            if (int rc = ensure(in_off, (size_t)(n + 1) * 8)) return rc;
            hipMemcpyAsync(in_bytes.p, bytes, (size_t)n_bytes, hipMemcpyHostToDevice, stream);
            hipMemcpyAsync(in_off.p, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, stream);
            d_bytes = (const uint8_t*)in_bytes.p;
            d_off = (const int64_t*)in_off.p;
        }
        JOut jo{};
        if (int rc = row_buffers(n, n_bytes, jo)) return rc;
        if (int rc = ensure(msg_err, (size_t)n)) return rc;
        if (int rc = ensure(aux, sizeof(JAux))) return rc;
        hipMemsetAsync(aux.p, 0, sizeof(JAux), stream);
        jo.err = (uint8_t*)msg_err.p;
        jo.rerr = jo.err;
        jo.rowbase = nullptr;
        jo.aux = (JAux*)aux.p;
        launch_decode(d_bytes, d_off, n, jo);
        int nb = (int)((n + kTile - 1) / kTile);
        if (int rc = ensure(cnt, (size_t)(nb + 1) * 8)) return rc;
        hipLaunchKernelGGL(k_ok_count, dim3(nb), dim3(kJBlock), 0, stream, (const uint8_t*)msg_err.p, n, (int64_t*)cnt.p);
        hipLaunchKernelGGL(k_scan_cnt, dim3(1), dim3(1024), 0, stream, (int64_t*)cnt.p, nb);
        int64_t ok = 0;
        JAux h_aux;
        hipMemcpyAsync(&ok, (int64_t*)cnt.p + nb, 8, hipMemcpyDeviceToHost, stream);
        hipMemcpyAsync(&h_aux, aux.p, sizeof h_aux, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "json decode kernel failed");
        int64_t R = n;              // decoded rows before the compaction
        int64_t failed = n - ok;    // messages that failed
        const uint8_t* rerr = (const uint8_t*)msg_err.p;
        if (h_aux.pending) {
            // some payload is a top-level array: rows per message, their offsets, and the row-based pass
            if (int rc = ensure(rowbase, (size_t)(n + 1) * 8 * 2)) return rc;
            int64_t* d_rows = (int64_t*)rowbase.p + (n + 1);
            hipLaunchKernelGGL(k_json_rows, dim3((unsigned)((n + kJBlock - 1) / kJBlock)), dim3(kJBlock), 0, stream, d_bytes,
                               d_off, n, d_rows);
            hipLaunchKernelGGL(k_rows_tile_sum, dim3(nb), dim3(kJBlock), 0, stream, (const int64_t*)d_rows, n, (int64_t*)cnt.p);
            hipLaunchKernelGGL(k_scan_cnt, dim3(1), dim3(1024), 0, stream, (int64_t*)cnt.p, nb);
            hipLaunchKernelGGL(k_rows_tile_scan, dim3(nb), dim3(kJBlock), 0, stream, (const int64_t*)d_rows, n,
                               (const int64_t*)cnt.p, nb, (int64_t*)rowbase.p);
            hipMemcpyAsync(&R, (int64_t*)rowbase.p + n, 8, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "json row count failed");
            if (int rc = row_buffers(R, n_bytes, jo)) return rc;
            if (int rc = ensure(row_err, (size_t)std::max<int64_t>(R, 1))) return rc;
            hipMemsetAsync(aux.p, 0, sizeof(JAux), stream);
            jo.rowbase = (const int64_t*)rowbase.p;
            jo.rerr = (uint8_t*)row_err.p;
            launch_decode(d_bytes, d_off, n, jo);
            rerr = (const uint8_t*)row_err.p;
            nb = (int)((std::max<int64_t>(R, 1) + kTile - 1) / kTile);
            if (int rc = ensure(cnt, (size_t)(nb + 1) * 8)) return rc;
            hipLaunchKernelGGL(k_ok_count, dim3(nb), dim3(kJBlock), 0, stream, rerr, R, (int64_t*)cnt.p);
            hipLaunchKernelGGL(k_scan_cnt, dim3(1), dim3(1024), 0, stream, (int64_t*)cnt.p, nb);
            std::vector<int64_t> rb((size_t)n + 1);
            h_err.resize((size_t)n);
            hipMemcpyAsync(&ok, (int64_t*)cnt.p + nb, 8, hipMemcpyDeviceToHost, stream);
            hipMemcpyAsync(&h_aux, aux.p, sizeof h_aux, hipMemcpyDeviceToHost, stream);
            hipMemcpyAsync(rb.data(), rowbase.p, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, stream);
            hipMemcpyAsync(h_err.data(), msg_err.p, (size_t)n, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "json decode kernel failed");
            h_rows_of.resize((size_t)n);
            failed = 0;
            for (int64_t i = 0; i < n; ++i) {
                h_rows_of[i] = h_err[i] ? 0 : rb[i + 1] - rb[i];
                failed += h_err[i] ? 1 : 0;
            }
        }
        last_ok = ok;
        st.messages += n;
        st.errors += failed;
        st.bytes += offsets && memory == EK_MEM_HOST ? (offsets[n] - offsets[0]) : 0;
        out->n_rows = ok;
        if (ok == R) {
            for (int c = 0; c < sch.n; ++c) {
                const bool list = sch.type[c] == EK_COL_LIST;
                out->columns[c] = list ? nullptr : raw_col[c].p;
                out->validity[c] = h_aux.nulls[c] ? (const uint8_t*)raw_valid[c].p : nullptr;   // no nil: no validity array
                str_off[c] = (const int64_t*)raw_soff[c].p;
                str_len[c] = (const int32_t*)raw_slen[c].p;
                if (list) { list_start[c] = (const int64_t*)raw_col[c].p; list_len[c] = (const int32_t*)raw_slen[c].p; }
            }
            return resolve_all(ok, false, d_bytes, memory == EK_MEM_HOST ? (const uint8_t*)bytes : nullptr, out);
        }
        // drop the rows of the messages that failed to decode (their errors are kept for ek_json_errors)
        if (int rc = ensure(pos, (size_t)R * 8)) return rc;
        hipLaunchKernelGGL(k_ok_pos, dim3(nb), dim3(kJBlock), 0, stream, rerr, R, (const int64_t*)cnt.p, (int64_t*)pos.p);
        const unsigned g = (unsigned)std::min<int64_t>(8192, (R + 255) / 256);
        for (int c = 0; c < sch.n; ++c) {
            const int es = sch.type[c] == EK_COL_U32 ? 4 : 8;
            const bool list = sch.type[c] == EK_COL_LIST;
            if (int rc = ensure(out_col[c], (size_t)std::max<int64_t>(ok, 1) * es)) return rc;
            if (int rc = ensure(out_valid[c], (size_t)std::max<int64_t>(ok, 1))) return rc;
            hipLaunchKernelGGL(k_compact_col, dim3(g), dim3(256), 0, stream, (const int64_t*)pos.p, R, raw_col[c].p, out_col[c].p, es);
            hipLaunchKernelGGL(k_compact_col, dim3(g), dim3(256), 0, stream, (const int64_t*)pos.p, R, raw_valid[c].p, out_valid[c].p, 1);
            out->columns[c] = list ? nullptr : out_col[c].p;
            out->validity[c] = h_aux.nulls[c] ? (const uint8_t*)out_valid[c].p : nullptr;
            if (sch.type[c] == EK_COL_STR) {
                if (int rc = ensure(out_soff[c], (size_t)std::max<int64_t>(ok, 1) * 8)) return rc;
                hipLaunchKernelGGL(k_compact_col, dim3(g), dim3(256), 0, stream, (const int64_t*)pos.p, R, raw_soff[c].p, out_soff[c].p, 8);
                str_off[c] = (const int64_t*)out_soff[c].p;
            }
            if (sch.type[c] == EK_COL_STR || list) {
                if (int rc = ensure(out_slen[c], (size_t)std::max<int64_t>(ok, 1) * 4)) return rc;
                hipLaunchKernelGGL(k_compact_col, dim3(g), dim3(256), 0, stream, (const int64_t*)pos.p, R, raw_slen[c].p, out_slen[c].p, 4);
                str_len[c] = (const int32_t*)out_slen[c].p;
            }
            if (list) { list_start[c] = (const int64_t*)out_col[c].p; list_len[c] = (const int32_t*)out_slen[c].p; }
        }
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "json compaction failed");
        return resolve_all(ok, true, d_bytes, memory == EK_MEM_HOST ? (const uint8_t*)bytes : nullptr, out);
    }

    // STRING column c of the decoded batch (rows n, hashes / validity / string refs at the given device arrays) ->
    // dense ids in id_col[c]. host_bytes: the payload on the host (EK_MEM_HOST) or null (d_bytes on the device only).
    int resolve_strings(int c, int64_t n, const int64_t* hash, const uint8_t* valid, const int64_t* soff, const int32_t* slen,
                        const uint8_t* d_bytes, const uint8_t* host_bytes, ek_batch* out) {
        StrDict& D = dict[c];
        if (int rc = ensure(id_col[c], (size_t)std::max<int64_t>(n, 1) * 4)) return rc;
        if (int rc = ensure(miss, (size_t)std::max<int64_t>(n, 1) * sizeof(MissRec))) return rc;
        if (int rc = ensure(n_miss, 8)) return rc;
        if (D.dirty) {
            if (int rc = ensure(tkey[c], D.hkey.size() * 8)) return rc;
            if (int rc = ensure(tval[c], D.hval.size() * 4)) return rc;
            if (int rc = ensure(tlen[c], D.hlen.size() * 4)) return rc;
            hipMemcpyAsync(tkey[c].p, D.hkey.data(), D.hkey.size() * 8, hipMemcpyHostToDevice, stream);
            hipMemcpyAsync(tval[c].p, D.hval.data(), D.hval.size() * 4, hipMemcpyHostToDevice, stream);
            hipMemcpyAsync(tlen[c].p, D.hlen.data(), D.hlen.size() * 4, hipMemcpyHostToDevice, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "string table upload failed");
            D.dirty = false;
        }
        hipMemsetAsync(n_miss.p, 0, 8, stream);
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256));
        hipLaunchKernelGGL(k_str_lookup, dim3(g), dim3(256), 0, stream, hash, soff, slen, valid, n,
                           (const uint64_t*)tkey[c].p, (const uint32_t*)tval[c].p, (const uint32_t*)tlen[c].p, D.bits,
                           (uint32_t*)id_col[c].p,
                           (MissRec*)miss.p, (unsigned long long*)n_miss.p);
        unsigned long long nm = 0;
        hipMemcpyAsync(&nm, n_miss.p, 8, hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "string lookup failed");
        out->columns[c] = id_col[c].p;
        if (nm == 0) return 0;
        std::vector<MissRec> mr((size_t)nm);
        hipMemcpyAsync(mr.data(), miss.p, (size_t)nm * sizeof(MissRec), hipMemcpyDeviceToHost, stream);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "string miss copy failed");
        std::sort(mr.begin(), mr.end(), [](const MissRec& a, const MissRec& b) { return a.row < b.row; });   // first-seen order
        std::vector<uint8_t> gathered;
        std::vector<int64_t> gpos((size_t)nm);
        const uint8_t* src = host_bytes;
        if (!src) {   // device payloads: gather the misses' bytes into one buffer, one copy back
            int64_t tot = 0;
            for (size_t k = 0; k < mr.size(); ++k) { gpos[k] = tot; tot += (mr[k].len & kStrNumber) ? 0 : (mr[k].len & ~kStrFlags); }
            if (int rc = ensure(gat_pos, mr.size() * 8)) return rc;
            if (int rc = ensure(gat_bytes, (size_t)std::max<int64_t>(tot, 1))) return rc;
            if (int rc = ensure(fix_rows, mr.size() * sizeof(MissRec))) return rc;
            hipMemcpyAsync(gat_pos.p, gpos.data(), mr.size() * 8, hipMemcpyHostToDevice, stream);
            hipMemcpyAsync(fix_rows.p, mr.data(), mr.size() * sizeof(MissRec), hipMemcpyHostToDevice, stream);
            const unsigned gg = (unsigned)std::max<size_t>(1, std::min<size_t>(8192, (mr.size() + 255) / 256));
            hipLaunchKernelGGL(k_str_gather, dim3(gg), dim3(256), 0, stream, d_bytes, (const MissRec*)fix_rows.p,
                               (const int64_t*)gat_pos.p, (int64_t)mr.size(), (uint8_t*)gat_bytes.p);
            gathered.resize((size_t)std::max<int64_t>(tot, 1));
            hipMemcpyAsync(gathered.data(), gat_bytes.p, (size_t)tot, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "string gather failed");
        }
        std::vector<int64_t> rows(mr.size());
        std::vector<uint32_t> ids(mr.size());
        std::string str;
        for (size_t k = 0; k < mr.size(); ++k) {
            const int32_t L = mr[k].len & ~kStrFlags;
            const uint8_t* b = src ? src + mr[k].off : gathered.data() + gpos[k];
            if (mr[k].len & kStrNumber) {
                double f;   // cast.ToStringAlways(float64): fmt's %v (converter.go:446-451)
                memcpy(&f, &mr[k].off, 8);
                str = ek::go_float(f);
            } else if (mr[k].len & EK_JSON_STR_ESCAPED) {
                str = json_unescape(b, L);
            } else {
                str.assign((const char*)b, (size_t)L);
            }
            auto it = D.ids.find(str);
            uint32_t id;
            if (it != D.ids.end()) {
                id = it->second;
            } else {
                if (D.values.size() >= 0xFFFFFFFFull) return fail(EK_ERR_NOMEM, "string dictionary full (2^32 - 1 strings)");
                id = (uint32_t)D.values.size();
                const uint64_t key = str_key(fnv1a64(str));
                auto hk = D.by_key.find(key);
                if (hk != D.by_key.end())
                    return fail(EK_ERR_UNSUPPORTED, "string hash collision: \"%s\" and \"%s\" share an FNV-1a 64 hash",
                                str.c_str(), D.values[hk->second].c_str());
                D.values.push_back(str);
                D.ids.emplace(str, id);
                D.insert(key, id);
            }
            rows[k] = mr[k].row;
            ids[k] = id;
        }
        if (int rc = ensure(fix_rows, rows.size() * 8)) return rc;
        if (int rc = ensure(fix_ids, ids.size() * 4)) return rc;
        hipMemcpyAsync(fix_rows.p, rows.data(), rows.size() * 8, hipMemcpyHostToDevice, stream);
        hipMemcpyAsync(fix_ids.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, stream);
        const unsigned gs = (unsigned)std::max<size_t>(1, std::min<size_t>(8192, (rows.size() + 255) / 256));
        hipLaunchKernelGGL(k_str_scatter, dim3(gs), dim3(256), 0, stream, (const int64_t*)fix_rows.p, (const uint32_t*)fix_ids.p,
                           (int64_t)rows.size(), (uint32_t*)id_col[c].p);
        if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "string id scatter failed");
        return 0;
    }
    int resolve_all(int64_t n, bool compacted, const uint8_t* d_bytes, const uint8_t* host_bytes, ek_batch* out) {
        for (int c = 0; c < sch.n; ++c) {
            if (sch.type[c] != EK_COL_STR) continue;
            const Buf& col = compacted ? out_col[c] : raw_col[c];
            const Buf& val = compacted ? out_valid[c] : raw_valid[c];
            if (int rc = resolve_strings(c, n, (const int64_t*)col.p, (const uint8_t*)val.p, str_off[c], str_len[c], d_bytes,
                                         host_bytes, out))
                return rc;
        }
        return 0;
    }

    int errors(int64_t* idx, uint8_t* code, int64_t cap, int64_t* n_out) {
        h_err.resize((size_t)last_n);
        if (last_n) {
            hipMemcpyAsync(h_err.data(), msg_err.p, (size_t)last_n, hipMemcpyDeviceToHost, stream);
            if (hipStreamSynchronize(stream) != hipSuccess) return fail(EK_ERR_DEVICE, "error copy failed");
        }
        int64_t k = 0;
        for (int64_t i = 0; i < last_n; ++i) {
            if (!h_err[i]) continue;
            if (k < cap) { if (idx) idx[k] = i; if (code) code[k] = h_err[i]; }
            k++;
        }
        *n_out = k;
        return 0;
    }
};

thread_local std::string g_json_create_error;

// Every entry point runs on the decoder's device and gives the calling thread its current device back (a Go node
// may call from any OS thread), like ek_engine.hip's DeviceGuard.
struct JsonDeviceGuard {
    int prev = -1;
    explicit JsonDeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) { prev = -1; return; }
        if (dev >= 0 && prev != dev) hipSetDevice(dev);
        else if (dev >= 0) prev = -1;
    }
    ~JsonDeviceGuard() { if (prev >= 0) hipSetDevice(prev); }
};

}  // namespace

extern "C" {

int ek_json_create(const ek_json_schema* schema, int device, void** out) {
    if (!out) return EK_ERR_INVALID;
    *out = nullptr;
    JsonDeviceGuard dg(-1);   // init selects `device`: the guard restores the caller's
    JsonDecoder* d = new (std::nothrow) JsonDecoder();
    if (!d) return EK_ERR_NOMEM;
    if (int rc = d->init(schema, device)) {
        g_json_create_error = d->err;
        delete d;
        return rc;
    }
    *out = d;
    return 0;
}

int ek_json_decode(void* h, const char* bytes, int64_t n_bytes, const int64_t* offsets, int64_t n_msgs, int32_t memory,
                   ek_batch* out) {
    if (!h) return EK_ERR_INVALID;
    JsonDeviceGuard dg(((JsonDecoder*)h)->dev);
    return ((JsonDecoder*)h)->decode(bytes, n_bytes, offsets, n_msgs, memory, out);
}

int ek_json_errors(void* h, int64_t* msg_index, uint8_t* code, int64_t cap, int64_t* n_errors) {
    if (!h || !n_errors) return EK_ERR_INVALID;
    JsonDeviceGuard dg(((JsonDecoder*)h)->dev);
    return ((JsonDecoder*)h)->errors(msg_index, code, cap, n_errors);
}

int ek_json_strings(void* h, int column, const int64_t** offsets, const int32_t** lengths) {
    if (!h || !offsets || !lengths) return EK_ERR_INVALID;
    JsonDecoder* d = (JsonDecoder*)h;
    if (column < 0 || column >= d->sch.n || d->sch.type[column] != EK_COL_STR) {
        d->err = "not a string column";
        return EK_ERR_INVALID;
    }
    *offsets = d->str_off[column];
    *lengths = d->str_len[column];
    return 0;
}

int ek_json_dict_size(void* h, int column, int64_t* n) {
    if (!h || !n) return EK_ERR_INVALID;
    JsonDecoder* d = (JsonDecoder*)h;
    if (column < 0 || column >= d->sch.n || d->sch.type[column] != EK_COL_STR) { d->err = "not a string column"; return EK_ERR_INVALID; }
    *n = (int64_t)d->dict[column].values.size();
    return 0;
}

int ek_json_dict_string(void* h, int column, uint32_t id, const char** s, int64_t* len) {
    if (!h || !s || !len) return EK_ERR_INVALID;
    JsonDecoder* d = (JsonDecoder*)h;
    if (column < 0 || column >= d->sch.n || d->sch.type[column] != EK_COL_STR) { d->err = "not a string column"; return EK_ERR_INVALID; }
    if (id >= d->dict[column].values.size()) { d->err = "string id out of range"; return EK_ERR_INVALID; }
    *s = d->dict[column].values[id].data();
    *len = (int64_t)d->dict[column].values[id].size();
    return 0;
}

int ek_json_list(void* h, int column, const int64_t** start, const int32_t** len, const int64_t** values,
                 const uint8_t** valid) {
    if (!h || !start || !len || !values || !valid) return EK_ERR_INVALID;
    JsonDecoder* d = (JsonDecoder*)h;
    if (column < 0 || column >= d->sch.n || d->sch.type[column] != EK_COL_LIST) { d->err = "not a LIST column"; return EK_ERR_INVALID; }
    *start = d->list_start[column];
    *len = d->list_len[column];
    *values = (const int64_t*)d->lval[column].p;
    *valid = (const uint8_t*)d->lvalid[column].p;
    return 0;
}

int ek_json_rows(void* h, const int64_t** rows_of, int64_t* n_msgs) {
    if (!h || !rows_of || !n_msgs) return EK_ERR_INVALID;
    JsonDecoder* d = (JsonDecoder*)h;
    JsonDeviceGuard dg(d->dev);
    if (d->h_rows_of.empty() && d->last_n > 0) {   // one row per decoded message
        d->h_err.resize((size_t)d->last_n);
        hipMemcpy(d->h_err.data(), d->msg_err.p, (size_t)d->last_n, hipMemcpyDeviceToHost);
        d->h_rows_of.resize((size_t)d->last_n);
        for (int64_t i = 0; i < d->last_n; ++i) d->h_rows_of[i] = d->h_err[i] ? 0 : 1;
    }
    *rows_of = d->h_rows_of.data();
    *n_msgs = d->last_n;
    return 0;
}

int ek_json_get_stats(void* h, ek_json_stats* out) {
    if (!h || !out) return EK_ERR_INVALID;
    *out = ((JsonDecoder*)h)->st;
    return 0;
}

const char* ek_json_last_error(void* h) { return h ? ((JsonDecoder*)h)->err.c_str() : g_json_create_error.c_str(); }

int ek_json_destroy(void* h) {
    if (!h) return 0;
    JsonDeviceGuard dg(((JsonDecoder*)h)->dev);
    delete (JsonDecoder*)h;
    return 0;
}

}  // extern "C"
