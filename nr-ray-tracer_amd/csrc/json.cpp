// JSON reader for scene files (`*.json`, app scene_config.rs:478-481).
//
// Number conversion follows serde_json 1.0.145's default (no
// `float_roundtrip`) path: the decimal significand is accumulated in a u64
// and then scaled by ONE multiplication/division with a power of ten, which
// is what `f64_from_parts` does (Cargo.lock:1366).  For every number in the
// reference's scene files this is the correctly-rounded value.
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "value.hpp"

namespace nrt {
namespace {

struct JsonReader {
    const std::string& t;
    size_t p = 0;
    int line = 1;

    explicit JsonReader(const std::string& s) : t(s) {}

    [[noreturn]] void fail(const std::string& msg) {
        throw ParseError(msg + " at line " + std::to_string(line));
    }
    void ws() {
        while (p < t.size()) {
            char c = t[p];
            if (c == '\n') { ++line; ++p; }
            else if (c == ' ' || c == '\t' || c == '\r') ++p;
            else break;
        }
    }
    bool eat(char c) {
        ws();
        if (p < t.size() && t[p] == c) { ++p; return true; }
        return false;
    }
    void expect(char c) {
        if (!eat(c)) fail(std::string("expected '") + c + "'");
    }
    static double pow10(int e) {
        static double table[309];
        static bool init = false;
        if (!init) {
            for (int k = 0; k < 309; ++k) {
                char buf[16];
                snprintf(buf, sizeof buf, "1e%d", k);
                table[k] = strtod(buf, nullptr);
            }
            init = true;
        }
        return table[e];
    }
    Value number() {
        size_t start = p;
        bool neg = false;
        if (t[p] == '-') { neg = true; ++p; }
        if (p >= t.size() || !isdigit((unsigned char)t[p])) fail("invalid number");
        uint64_t sig = 0;
        bool overflow = false, is_float = false;
        int exp10 = 0;
        auto digit = [&](int d, bool frac) {
            if (!overflow && sig <= (UINT64_MAX - (uint64_t)d) / 10) {
                sig = sig * 10 + (uint64_t)d;
                if (frac) --exp10;
            } else {
                overflow = true;
                if (!frac) ++exp10;
            }
        };
        if (t[p] == '0') { ++p; }
        else while (p < t.size() && isdigit((unsigned char)t[p])) digit(t[p++] - '0', false);
        if (p < t.size() && t[p] == '.') {
            is_float = true;
            ++p;
            if (p >= t.size() || !isdigit((unsigned char)t[p])) fail("invalid number");
            while (p < t.size() && isdigit((unsigned char)t[p])) digit(t[p++] - '0', true);
        }
        if (p < t.size() && (t[p] == 'e' || t[p] == 'E')) {
            is_float = true;
            ++p;
            int esign = 1, e = 0;
            if (t[p] == '+') ++p;
            else if (t[p] == '-') { esign = -1; ++p; }
            if (p >= t.size() || !isdigit((unsigned char)t[p])) fail("invalid number");
            while (p < t.size() && isdigit((unsigned char)t[p])) {
                if (e < 100000) e = e * 10 + (t[p] - '0');
                ++p;
            }
            exp10 += esign * e;
        }
        Value v;
        if (!is_float && !overflow && (neg ? sig <= (uint64_t)INT64_MAX + 1 : sig <= (uint64_t)INT64_MAX)) {
            v.kind = Value::Int;
            v.i = neg ? (int64_t)(0 - sig) : (int64_t)sig;
            return v;
        }
        v.kind = Value::Float;
        if (overflow || exp10 > 308 || exp10 < -308) {
            // Outside the fast path: fall back to a correctly rounded parse.
            v.f = strtod(t.substr(start, p - start).c_str(), nullptr);
            return v;
        }
        double f = (double)sig;
        if (exp10 >= 0) {
            f *= pow10(exp10);
            if (std::isinf(f)) fail("number out of range");
        } else {
            f /= pow10(-exp10);
        }
        v.f = neg ? -f : f;
        return v;
    }
    void utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) out += (char)cp;
        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 63)); }
        else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 63));
            out += (char)(0x80 | (cp & 63));
        } else {
            out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 63));
            out += (char)(0x80 | ((cp >> 6) & 63)); out += (char)(0x80 | (cp & 63));
        }
    }
    uint32_t hex4() {
        if (p + 4 > t.size()) fail("bad \\u escape");
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            char c = t[p++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else fail("bad \\u escape");
        }
        return v;
    }
    std::string string() {
        expect('"');
        std::string out;
        while (true) {
            if (p >= t.size()) fail("unterminated string");
            char c = t[p++];
            if (c == '"') break;
            if (c == '\\') {
                char e = t[p++];
                switch (e) {
                    case '"': out += '"'; break;
                    case '\\': out += '\\'; break;
                    case '/': out += '/'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'n': out += '\n'; break;
                    case 'r': out += '\r'; break;
                    case 't': out += '\t'; break;
                    case 'u': {
                        uint32_t cp = hex4();
                        if (cp >= 0xD800 && cp < 0xDC00 && p + 6 <= t.size() && t[p] == '\\' && t[p + 1] == 'u') {
                            p += 2;
                            uint32_t lo = hex4();
                            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                        }
                        utf8(out, cp);
                        break;
                    }
                    default: fail("bad escape");
                }
            } else {
                if ((unsigned char)c < 0x20) fail("control character in string");
                out += c;
            }
        }
        return out;
    }
    Value value(int depth) {
        if (depth > 256) fail("nesting too deep");
        ws();
        if (p >= t.size()) fail("unexpected end of input");
        char c = t[p];
        if (c == '{') {
            ++p;
            Value v = Value::make(Value::Table);
            if (eat('}')) return v;
            do {
                ws();
                std::string k = string();
                expect(':');
                Value child = value(depth + 1);
                if (Value* prev = v.get_mut(k)) *prev = std::move(child);
                else v.insert(k, std::move(child));
            } while (eat(','));
            expect('}');
            return v;
        }
        if (c == '[') {
            ++p;
            Value v = Value::make(Value::Array);
            if (eat(']')) return v;
            do { v.arr.push_back(value(depth + 1)); } while (eat(','));
            expect(']');
            return v;
        }
        if (c == '"') { Value v = Value::make(Value::String); v.s = string(); return v; }
        if (t.compare(p, 4, "true") == 0) { p += 4; Value v = Value::make(Value::Bool); v.b = true; return v; }
        if (t.compare(p, 5, "false") == 0) { p += 5; return Value::make(Value::Bool); }
        if (t.compare(p, 4, "null") == 0) { p += 4; return Value::make(Value::Null); }
        if (c == '-' || isdigit((unsigned char)c)) return number();
        fail(std::string("unexpected character '") + c + "'");
    }
};

}  // namespace

Value parse_json(const std::string& text) {
    JsonReader r(text);
    Value v = r.value(0);
    r.ws();
    if (r.p != text.size()) r.fail("trailing characters");
    return v;
}

}  // namespace nrt
