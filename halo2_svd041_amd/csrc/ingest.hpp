// Ingest of the example's input file data/matrix.in (examples/svd_example.rs:
// 326-330: `serde_json::from_str` into { m: Vec<Vec<f64>>, u, v, d: Vec<f64> }),
// written by input-creator.py:23-44 (json.dump of Python floats).
//
// Two float parses:
//   kParseSerde   serde_json 1.0's default path (no `float_roundtrip`): the
//                 decimal significand as u64 -> f64, then one multiply / divide
//                 by the f64 power-of-ten table entry 10^|e| (1e308 steps past
//                 the table); differs from correct rounding by 1 ulp on ~10 % of
//                 input-creator values, which changes quantized cells.
//   kParseCorrect correctly rounded (strtod).
// Significands beyond u64 (not produced by input-creator) are rejected rather
// than guessed. Host code: the text is a few tens of MB at 1024^2.
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

namespace svdw_ingest {

enum { kParseSerde = 0, kParseCorrect = 1 };

struct Array {
    std::vector<double> v;
    uint32_t rows = 0, cols = 0;   // 1-D: rows = 0, cols = length
    bool seen = false;
};
struct SvdInput {
    Array m, u, v, d;
};

class Parser {
  public:
    Parser(const char* s, uint64_t n, int mode) : b_(s), p_(s), e_(s + n), mode_(mode) {}

    bool parse(SvdInput& out, std::string& err) {
        try {
            ws();
            expect('{');
            ws();
            if (peek() == '}') { ++p_; return finish(out, err); }
            for (;;) {
                ws();
                const std::string key = str();
                ws();
                expect(':');
                ws();
                Array* dst = key == "m" ? &out.m : key == "u" ? &out.u : key == "v" ? &out.v
                           : key == "d" ? &out.d : nullptr;
                if (dst) {
                    if (dst->seen) throw std::string("duplicate key \"" + key + "\"");
                    array(*dst);
                } else {
                    skip_value();
                }
                ws();
                if (peek() == ',') { ++p_; continue; }
                expect('}');
                break;
            }
            ws();
            if (p_ != e_) throw std::string("trailing characters after the JSON object");
            return finish(out, err);
        } catch (const std::string& msg) {
            err = msg + " (at byte " + std::to_string(p_ - b_) + ")";
            return false;
        }
    }

  private:
    const char* b_;
    const char* p_;
    const char* e_;
    int mode_;

    bool finish(SvdInput& out, std::string& err) {
        for (auto* a : {&out.m, &out.u, &out.v, &out.d})
            if (!a->seen) { err = "missing one of the keys m, u, v, d"; return false; }
        return true;
    }
    char peek() const { return p_ < e_ ? *p_ : '\0'; }
    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
    }
    void expect(char c) {
        if (p_ >= e_ || *p_ != c) throw std::string("expected '") + c + "'";
        ++p_;
    }
    std::string str() {
        expect('"');
        std::string s;
        while (p_ < e_ && *p_ != '"') {
            if (*p_ == '\\') {
                ++p_;
                if (p_ >= e_) break;
            }
            s.push_back(*p_++);
        }
        expect('"');
        return s;
    }
    void skip_value() {
        ws();
        const char c = peek();
        if (c == '"') { str(); return; }
        if (c == '[' || c == '{') {
            const char open = c, close = c == '[' ? ']' : '}';
            int depth = 0;
            do {
                if (p_ >= e_) throw std::string("unterminated value");
                if (*p_ == '"') { str(); continue; }
                if (*p_ == open) ++depth;
                if (*p_ == close) --depth;
                ++p_;
            } while (depth > 0);
            return;
        }
        while (p_ < e_ && *p_ != ',' && *p_ != '}' && *p_ != ']') ++p_;
    }
    // [n, n, ...] or [[n, ...], [n, ...], ...] (rectangular)
    void array(Array& a) {
        a.seen = true;
        expect('[');
        ws();
        if (peek() == ']') { ++p_; return; }
        if (peek() == '[') {
            for (;;) {
                ws();
                expect('[');
                uint32_t cols = 0;
                ws();
                if (peek() != ']') {
                    for (;;) {
                        ws();
                        a.v.push_back(number());
                        ++cols;
                        ws();
                        if (peek() == ',') { ++p_; continue; }
                        break;
                    }
                }
                expect(']');
                if (a.rows && cols != a.cols) throw std::string("ragged matrix rows");
                a.cols = cols;
                ++a.rows;
                ws();
                if (peek() == ',') { ++p_; continue; }
                break;
            }
        } else {
            for (;;) {
                ws();
                a.v.push_back(number());
                ws();
                if (peek() == ',') { ++p_; continue; }
                break;
            }
            a.cols = (uint32_t)a.v.size();
        }
        ws();
        expect(']');
    }
    double number() {
        const char* s = p_;
        if (p_ < e_ && *p_ == '-') ++p_;
        const char* digits = p_;
        while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
        if (p_ == digits) throw std::string("expected a number");
        const char* int_end = p_;
        const char* frac = nullptr;
        const char* frac_end = nullptr;
        if (p_ < e_ && *p_ == '.') {
            frac = ++p_;
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
            frac_end = p_;
            if (frac == frac_end) throw std::string("expected fraction digits");
        }
        int64_t exp10 = 0;
        if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
            ++p_;
            bool eneg = false;
            if (p_ < e_ && (*p_ == '+' || *p_ == '-')) eneg = *p_++ == '-';
            const char* ed = p_;
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') {
                if (exp10 < 100000) exp10 = exp10 * 10 + (*p_ - '0');
                ++p_;
            }
            if (p_ == ed) throw std::string("expected exponent digits");
            if (eneg) exp10 = -exp10;
        }
        if (mode_ == kParseCorrect) {
            const std::string tok(s, (size_t)(p_ - s));
            return strtod(tok.c_str(), nullptr);
        }
        // serde_json default: u64 significand of all digits, then f64_from_parts
        const bool neg = *s == '-';
        uint64_t sig = 0;
        auto acc = [&](const char* a, const char* b) {
            for (const char* q = a; q < b; ++q) {
                const uint64_t dgt = (uint64_t)(*q - '0');
                if (sig > (UINT64_MAX - dgt) / 10)
                    throw std::string("significand beyond u64 (serde's overflow path is not emulated)");
                sig = sig * 10 + dgt;
            }
        };
        acc(digits, int_end);
        if (frac) acc(frac, frac_end);
        int64_t e = exp10 - (frac ? (int64_t)(frac_end - frac) : 0);
        double f = (double)sig;
        for (;;) {
            const int64_t ae = e < 0 ? -e : e;
            if (ae <= 308) {
                const double pw = pow10_table(ae);
                f = e >= 0 ? f * pw : f / pw;
                break;
            }
            if (f == 0.0) break;
            if (e >= 0) throw std::string("number out of range");
            f /= 1e308;
            e += 308;
        }
        return neg ? -f : f;
    }
    // 10^k, k <= 308, as the correctly rounded f64 literal (serde's POW10 table)
    static double pow10_table(int64_t k) {
        static const std::vector<double> t = [] {
            std::vector<double> v(309);
            char buf[16];
            for (int i = 0; i <= 308; ++i) {
                snprintf(buf, sizeof buf, "1e%d", i);
                v[i] = strtod(buf, nullptr);
            }
            return v;
        }();
        return t[(size_t)k];
    }
};

}  // namespace svdw_ingest
