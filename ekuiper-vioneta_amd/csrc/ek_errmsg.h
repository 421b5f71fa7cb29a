// ek_errmsg.h — host-side text of a window's WHERE / HAVING error (ek_window_error).
//
// The device kernels only flag a window (win_status) and record a witness: the window's first row whose WHERE failed
// to evaluate, or a group whose HAVING did, with the values the program reads (the row's columns / the group's
// aggregate slots). This file re-runs the program over those values on the host — the same postfix ISA and the same
// rules as the device interpreter (ek_device.h eval_prog / simple_eval, which restate valuer.go:574-1000) — and prints
// the error the reference's operator returns:
//   FilterOp  (filter_operator.go:45-58):  "run Where error: %s" | "... invalid condition that returns non-bool value %T(%v)"
//   HavingOp  (having_operator.go:45-55):  "run Having error: %s" | the same non-bool text
// with %s one of valuer.go's texts: "divided by zero" (:897-979) or invalidOpError (:1243-1245)
// "invalid operation %T(%v) %s %T(%v)" with ast.Tokens spellings (pkg/ast/token.go:135-193).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/ekgpu.h"

namespace ek {

struct HVal {
    enum : int { NUL = 0, BOOL = 1, I64 = 2, F64 = 3, ERR = 4 };
    int tag = NUL;
    int64_t i = 0;
    double f = 0.0;
    std::string err;   // ERR: the valuer's message
};

// Go's %v of a float64: fmt prints it as strconv.FormatFloat(f, 'g', -1, 64) — the shortest digits that round-trip,
// in %e form (d.ddde±XX) when the decimal exponent is < -4 or >= 6 (strconv/ftoa.go formatDigits: eprec = 6 for the
// shortest form), %f form otherwise: 2.5, 100000, 1e+06, 1.234567e+06, 1e-05.
inline std::string go_float(double v) {
    if (std::isnan(v)) return "NaN";
    if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
    if (v == 0) return std::signbit(v) ? "-0" : "0";
    // shortest round-trip decimal digits: d1.d2d3...e<exp10>
    char buf[64];
    int prec = 1;
    for (; prec <= 17; ++prec) {
        std::snprintf(buf, sizeof buf, "%.*e", prec - 1, v);
        if (std::strtod(buf, nullptr) == v) break;
    }
    std::string s(buf);
    const bool neg = s[0] == '-';
    if (neg) s.erase(0, 1);
    const size_t epos = s.find('e');
    const int exp10 = std::atoi(s.c_str() + epos + 1);
    std::string digs;
    for (size_t k = 0; k < epos; ++k)
        if (s[k] != '.') digs.push_back(s[k]);
    while (digs.size() > 1 && digs.back() == '0') digs.pop_back();
    const int nd = (int)digs.size();
    const int dp = exp10 + 1;   // decimal point position (digits before it)
    const int x = dp - 1;
    std::string out = neg ? "-" : "";
    if (x < -4 || x >= 6) {
        // %e: d[.ddd]e±XX (at least two exponent digits)
        out += digs[0];
        if (nd > 1) { out += '.'; out += digs.substr(1); }
        char eb[16];
        std::snprintf(eb, sizeof eb, "e%c%02d", x < 0 ? '-' : '+', x < 0 ? -x : x);
        out += eb;
        return out;
    }
    // %f with the shortest digits
    if (dp <= 0) {
        out += "0.";
        out += std::string((size_t)(-dp), '0');
        out += digs;
    } else if (dp >= nd) {
        out += digs;
        out += std::string((size_t)(dp - nd), '0');
    } else {
        out += digs.substr(0, (size_t)dp);
        out += '.';
        out += digs.substr((size_t)dp);
    }
    return out;
}

// %T(%v)
inline std::string go_tv(const HVal& v) {
    switch (v.tag) {
    case HVal::BOOL: return std::string("bool(") + (v.i ? "true" : "false") + ")";
    case HVal::I64: return "int64(" + std::to_string((long long)v.i) + ")";
    case HVal::F64: return "float64(" + go_float(v.f) + ")";
    default: return "<nil>(<nil>)";
    }
}

inline const char* go_token(int op) {
    switch (op) {
    case EK_OP_EQ: return "=";
    case EK_OP_NEQ: return "!=";
    case EK_OP_LT: return "<";
    case EK_OP_LTE: return "<=";
    case EK_OP_GT: return ">";
    case EK_OP_GTE: return ">=";
    case EK_OP_AND: return "AND";
    case EK_OP_OR: return "OR";
    case EK_OP_ADD: return "+";
    case EK_OP_SUB: return "-";
    case EK_OP_MUL: return "*";
    case EK_OP_DIV: return "/";
    case EK_OP_MOD: return "%";
    default: return "?";
    }
}

inline HVal hv_bool(bool b) { HVal v; v.tag = HVal::BOOL; v.i = b; return v; }
inline HVal hv_err(std::string m) { HVal v; v.tag = HVal::ERR; v.err = std::move(m); return v; }
inline HVal hv_invalid(const HVal& l, int op, const HVal& r) {   // valuer.go:1243-1245
    return hv_err("invalid operation " + go_tv(l) + " " + go_token(op) + " " + go_tv(r));
}

// valuer.go:823-1000 SimpleDataEval over non-error operands (same branches as ek_device.h simple_eval)
inline HVal h_simple_eval(const HVal& l, const HVal& r, int op) {
    if (l.tag == HVal::NUL || r.tag == HVal::NUL) {
        if (op >= EK_OP_EQ && op <= EK_OP_OR) return hv_bool(false);
        return HVal{};
    }
    if (l.tag == HVal::BOOL) {
        if (r.tag != HVal::BOOL) return hv_invalid(l, op, r);
        switch (op) {
        case EK_OP_AND: return hv_bool(l.i && r.i);
        case EK_OP_OR: return hv_bool(l.i || r.i);
        case EK_OP_EQ: return hv_bool(l.i == r.i);
        case EK_OP_NEQ: return hv_bool(l.i != r.i);
        default: return hv_invalid(l, op, r);
        }
    }
    if (r.tag == HVal::BOOL) return hv_invalid(l, op, r);   // a number lhs against a bool (:872-873, :1042-1043)
    if (l.tag == HVal::F64 || r.tag == HVal::F64) {
        // an int64 lhs against a float64 rhs is converted first (:911-912), a float64 lhs takes the rhs as float (:863-868)
        HVal lf; lf.tag = HVal::F64; lf.f = l.tag == HVal::F64 ? l.f : (double)l.i;
        HVal rf; rf.tag = HVal::F64; rf.f = r.tag == HVal::F64 ? r.f : (double)r.i;
        const double a = lf.f, c = rf.f;
        HVal o; o.tag = HVal::F64;
        switch (op) {
        case EK_OP_EQ: return hv_bool(a == c);
        case EK_OP_NEQ: return hv_bool(a != c);
        case EK_OP_LT: return hv_bool(a < c);
        case EK_OP_LTE: return hv_bool(a <= c);
        case EK_OP_GT: return hv_bool(a > c);
        case EK_OP_GTE: return hv_bool(a >= c);
        case EK_OP_ADD: o.f = a + c; return o;
        case EK_OP_SUB: o.f = a - c; return o;
        case EK_OP_MUL: o.f = a * c; return o;
        case EK_OP_DIV: if (c == 0) return hv_err("divided by zero"); o.f = a / c; return o;
        case EK_OP_MOD: if (c == 0) return hv_err("divided by zero"); o.f = std::fmod(a, c); return o;
        default: return hv_invalid(lf, op, rf);
        }
    }
    const int64_t a = l.i, c = r.i;
    HVal o; o.tag = HVal::I64;
    switch (op) {
    case EK_OP_EQ: return hv_bool(a == c);
    case EK_OP_NEQ: return hv_bool(a != c);
    case EK_OP_LT: return hv_bool(a < c);
    case EK_OP_LTE: return hv_bool(a <= c);
    case EK_OP_GT: return hv_bool(a > c);
    case EK_OP_GTE: return hv_bool(a >= c);
    case EK_OP_ADD: o.i = (int64_t)((uint64_t)a + (uint64_t)c); return o;
    case EK_OP_SUB: o.i = (int64_t)((uint64_t)a - (uint64_t)c); return o;
    case EK_OP_MUL: o.i = (int64_t)((uint64_t)a * (uint64_t)c); return o;
    case EK_OP_DIV: if (c == 0) return hv_err("divided by zero"); o.i = (a == INT64_MIN && c == -1) ? a : a / c; return o;
    case EK_OP_MOD: if (c == 0) return hv_err("divided by zero"); o.i = c == -1 ? 0 : a % c; return o;
    default: return hv_invalid(l, op, r);
    }
}

// evalBinaryExpr (valuer.go:574-601): an lhs error wins, then the AND/OR short cut, then an rhs error
template <typename COLF, typename AGGF>
inline HVal h_eval_prog(const ek_instr* prog, int n, COLF colf, AGGF aggf) {
    HVal st[EK_MAX_PROG + 1];
    int sp = 0;
    for (int k = 0; k < n; ++k) {
        const int op = prog[k].op;
        if (op == EK_OP_COL) st[sp++] = colf(prog[k].arg);
        else if (op == EK_OP_AGG) st[sp++] = aggf(prog[k].arg);
        else if (op == EK_OP_CONST_I64) { HVal v; v.tag = HVal::I64; v.i = prog[k].i64; st[sp++] = v; }
        else if (op == EK_OP_CONST_F64) { HVal v; v.tag = HVal::F64; v.f = prog[k].f64; st[sp++] = v; }
        else if (op == EK_OP_CONST_BOOL) st[sp++] = hv_bool(prog[k].i64 != 0);
        else {
            if (sp < 2) return hv_err("malformed program");
            HVal r = std::move(st[--sp]);
            HVal l = std::move(st[--sp]);
            HVal res;
            if (l.tag == HVal::ERR) res = std::move(l);
            else if (op == EK_OP_AND && l.tag == HVal::BOOL && !l.i) res = hv_bool(false);
            else if (op == EK_OP_OR && l.tag == HVal::BOOL && l.i) res = hv_bool(true);
            else if (r.tag == HVal::ERR) res = std::move(r);
            else res = h_simple_eval(l, r, op);
            st[sp++] = std::move(res);
        }
    }
    return sp ? st[sp - 1] : HVal{};
}

// The operator's error text for a condition result, or "" when the result is not an error for that operator
// (WHERE: nil / bool are fine; HAVING: only bool is, nil is "non-bool value <nil>(<nil>)").
inline std::string condition_error(const char* prefix, const HVal& v, bool nil_ok) {
    if (v.tag == HVal::ERR) return std::string(prefix) + v.err;
    if (v.tag == HVal::BOOL || (nil_ok && v.tag == HVal::NUL)) return "";
    return std::string(prefix) + "invalid condition that returns non-bool value " + go_tv(v);
}

}  // namespace ek
