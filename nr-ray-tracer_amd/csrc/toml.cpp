// TOML reader for scene files (`*.toml`, app scene_config.rs:482-485).
//
// Covers what the reference's scenes and the `create` generators emit
// (toml 0.9.8, Cargo.lock:1588): tables, dotted table headers, arrays of
// tables, dotted keys, inline tables (newlines tolerated, as in noise.toml:1-26),
// heterogeneous multi-line arrays, basic/literal/multi-line strings,
// integers (dec/hex/oct/bin, underscores), floats (incl. inf/nan), booleans.
// Floats are converted with strtod (correctly rounded, like Rust's
// `str::parse::<f64>` used by the toml crate).  Date-times are rejected.
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "value.hpp"

namespace nrt {
namespace {

struct TomlReader {
    const std::string& t;
    size_t p = 0;
    int line = 1;
    Value root = Value::make(Value::Table);

    explicit TomlReader(const std::string& s) : t(s) {}

    [[noreturn]] void fail(const std::string& msg) {
        throw ParseError("TOML: " + msg + " at line " + std::to_string(line));
    }
    bool at_end() const { return p >= t.size(); }
    char cur() const { return p < t.size() ? t[p] : '\0'; }

    void skip_inline_ws() {
        while (!at_end() && (t[p] == ' ' || t[p] == '\t')) ++p;
    }
    void skip_comment() {
        if (cur() == '#')
            while (!at_end() && t[p] != '\n') ++p;
    }
    // whitespace, newlines and comments (inside arrays / inline tables)
    void skip_all_ws() {
        while (!at_end()) {
            char c = t[p];
            if (c == ' ' || c == '\t' || c == '\r') ++p;
            else if (c == '\n') { ++line; ++p; }
            else if (c == '#') skip_comment();
            else break;
        }
    }
    void end_of_line() {
        skip_inline_ws();
        skip_comment();
        if (cur() == '\r') ++p;
        if (at_end()) return;
        if (cur() != '\n') fail("expected end of line");
        ++p;
        ++line;
    }

    static bool bare_char(char c) {
        return isalnum((unsigned char)c) || c == '_' || c == '-';
    }

    std::string key_part() {
        skip_inline_ws();
        char c = cur();
        if (c == '"') return basic_string();
        if (c == '\'') return literal_string();
        size_t s = p;
        while (!at_end() && bare_char(t[p])) ++p;
        if (s == p) fail("expected a key");
        return t.substr(s, p - s);
    }
    std::vector<std::string> dotted_key() {
        std::vector<std::string> parts;
        parts.push_back(key_part());
        skip_inline_ws();
        while (cur() == '.') {
            ++p;
            parts.push_back(key_part());
            skip_inline_ws();
        }
        return parts;
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
    uint32_t hexn(int n) {
        uint32_t v = 0;
        for (int k = 0; k < n; ++k) {
            if (at_end()) fail("bad unicode escape");
            char c = t[p++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else fail("bad unicode escape");
        }
        return v;
    }
    void escape(std::string& out) {
        char e = t[p++];
        switch (e) {
            case 'b': out += '\b'; break;
            case 't': out += '\t'; break;
            case 'n': out += '\n'; break;
            case 'f': out += '\f'; break;
            case 'r': out += '\r'; break;
            case 'e': out += '\x1b'; break;
            case '"': out += '"'; break;
            case '\\': out += '\\'; break;
            case 'u': utf8(out, hexn(4)); break;
            case 'U': utf8(out, hexn(8)); break;
            default: fail("bad escape");
        }
    }
    std::string basic_string() {
        if (t.compare(p, 3, "\"\"\"") == 0) {
            p += 3;
            if (cur() == '\r') ++p;
            if (cur() == '\n') { ++p; ++line; }
            std::string out;
            while (true) {
                if (at_end()) fail("unterminated string");
                if (t.compare(p, 3, "\"\"\"") == 0) {
                    p += 3;
                    while (cur() == '"') { out += '"'; ++p; }
                    return out;
                }
                char c = t[p++];
                if (c == '\\') {
                    // line-ending backslash trims following whitespace
                    size_t q = p;
                    while (q < t.size() && (t[q] == ' ' || t[q] == '\t' || t[q] == '\r')) ++q;
                    if (q < t.size() && t[q] == '\n') {
                        p = q;
                        while (!at_end() && (t[p] == ' ' || t[p] == '\t' || t[p] == '\r' || t[p] == '\n')) {
                            if (t[p] == '\n') ++line;
                            ++p;
                        }
                    } else {
                        escape(out);
                    }
                } else {
                    if (c == '\n') ++line;
                    out += c;
                }
            }
        }
        ++p;  // opening quote
        std::string out;
        while (true) {
            if (at_end() || t[p] == '\n') fail("unterminated string");
            char c = t[p++];
            if (c == '"') return out;
            if (c == '\\') escape(out);
            else out += c;
        }
    }
    std::string literal_string() {
        if (t.compare(p, 3, "'''") == 0) {
            p += 3;
            if (cur() == '\r') ++p;
            if (cur() == '\n') { ++p; ++line; }
            size_t e = t.find("'''", p);
            if (e == std::string::npos) fail("unterminated string");
            while (e + 3 < t.size() && t[e + 3] == '\'') ++e;
            std::string out = t.substr(p, e - p);
            for (char c : out) if (c == '\n') ++line;
            p = e + 3;
            return out;
        }
        ++p;
        size_t e = t.find('\'', p);
        size_t nl = t.find('\n', p);
        if (e == std::string::npos || (nl != std::string::npos && nl < e)) fail("unterminated string");
        std::string out = t.substr(p, e - p);
        p = e + 1;
        return out;
    }

    Value number_or_bool() {
        if (t.compare(p, 4, "true") == 0 && !bare_char(p + 4 < t.size() ? t[p + 4] : ' ')) {
            p += 4;
            Value v = Value::make(Value::Bool); v.b = true; return v;
        }
        if (t.compare(p, 5, "false") == 0 && !bare_char(p + 5 < t.size() ? t[p + 5] : ' ')) {
            p += 5;
            return Value::make(Value::Bool);
        }
        size_t s = p;
        while (!at_end() && (isalnum((unsigned char)t[p]) || t[p] == '_' || t[p] == '+' || t[p] == '-' ||
                             t[p] == '.' || t[p] == ':'))
            ++p;
        std::string tok = t.substr(s, p - s);
        if (tok.empty()) fail("expected a value");
        std::string clean;
        for (char c : tok) if (c != '_') clean += c;
        Value v;
        std::string body = clean;
        bool neg = false;
        if (!body.empty() && (body[0] == '+' || body[0] == '-')) { neg = body[0] == '-'; body = body.substr(1); }
        if (body == "inf" || body == "nan") {
            v.kind = Value::Float;
            v.f = body == "inf" ? INFINITY : NAN;
            if (neg) v.f = -v.f;
            return v;
        }
        if (body.size() > 2 && body[0] == '0' && (body[1] == 'x' || body[1] == 'o' || body[1] == 'b')) {
            int base = body[1] == 'x' ? 16 : body[1] == 'o' ? 8 : 2;
            char* end = nullptr;
            unsigned long long u = strtoull(body.c_str() + 2, &end, base);
            if (*end != '\0') fail("invalid integer '" + tok + "'");
            v.kind = Value::Int;
            v.i = (int64_t)u;
            return v;
        }
        if (tok.find(':') != std::string::npos || (body.size() >= 10 && body[4] == '-' && body[7] == '-'))
            fail("date-time values are not supported");
        bool is_float = body.find_first_of(".eE") != std::string::npos;
        char* end = nullptr;
        if (is_float) {
            v.kind = Value::Float;
            v.f = strtod(clean.c_str(), &end);
        } else {
            v.kind = Value::Int;
            errno = 0;
            v.i = strtoll(clean.c_str(), &end, 10);
            if (errno == ERANGE) fail("integer out of range");
        }
        if (end == nullptr || *end != '\0') fail("invalid value '" + tok + "'");
        return v;
    }

    Value value(int depth) {
        if (depth > 128) fail("nesting too deep");
        skip_inline_ws();
        char c = cur();
        if (c == '"') { Value v = Value::make(Value::String); v.s = basic_string(); return v; }
        if (c == '\'') { Value v = Value::make(Value::String); v.s = literal_string(); return v; }
        if (c == '[') {
            ++p;
            Value v = Value::make(Value::Array);
            v.toml_inline = true;
            while (true) {
                skip_all_ws();
                if (cur() == ']') { ++p; break; }
                v.arr.push_back(value(depth + 1));
                skip_all_ws();
                if (cur() == ',') { ++p; continue; }
                if (cur() == ']') { ++p; break; }
                fail("expected ',' or ']' in array");
            }
            return v;
        }
        if (c == '{') {
            ++p;
            Value v = Value::make(Value::Table);
            v.toml_inline = true;
            while (true) {
                skip_all_ws();
                if (cur() == '}') { ++p; break; }
                std::vector<std::string> key = dotted_key();
                skip_inline_ws();
                if (cur() != '=') fail("expected '=' in inline table");
                ++p;
                Value child = value(depth + 1);
                assign(v, key, std::move(child));
                skip_all_ws();
                if (cur() == ',') { ++p; continue; }
                if (cur() == '}') { ++p; break; }
                fail("expected ',' or '}' in inline table");
            }
            return v;
        }
        return number_or_bool();
    }

    // Assign `key = value` relative to table `tbl` (dotted keys create tables).
    void assign(Value& tbl, const std::vector<std::string>& key, Value v) {
        Value* cur_t = &tbl;
        for (size_t k = 0; k + 1 < key.size(); ++k) {
            Value* next = cur_t->get_mut(key[k]);
            if (!next) next = &cur_t->insert(key[k], Value::make(Value::Table));
            else if (next->kind != Value::Table || next->toml_inline) fail("key '" + key[k] + "' is not a table");
            cur_t = next;
        }
        if (cur_t->get(key.back())) fail("duplicate key '" + key.back() + "'");
        cur_t->insert(key.back(), std::move(v));
    }

    // Navigate a header path; arrays of tables resolve to their last element.
    Value* navigate(const std::vector<std::string>& path, size_t upto) {
        Value* cur_t = &root;
        for (size_t k = 0; k < upto; ++k) {
            Value* next = cur_t->get_mut(path[k]);
            if (!next) next = &cur_t->insert(path[k], Value::make(Value::Table));
            if (next->kind == Value::Array) {
                if (!next->toml_aot || next->arr.empty()) fail("cannot extend static array '" + path[k] + "'");
                next = &next->arr.back();
            }
            if (next->kind != Value::Table || next->toml_inline) fail("'" + path[k] + "' is not a table");
            cur_t = next;
        }
        return cur_t;
    }

    void parse() {
        Value* current = &root;
        while (true) {
            skip_all_ws();
            if (at_end()) break;
            if (cur() == '[') {
                bool aot = t.compare(p, 2, "[[") == 0;
                p += aot ? 2 : 1;
                std::vector<std::string> path = dotted_key();
                skip_inline_ws();
                if (aot) {
                    if (t.compare(p, 2, "]]") != 0) fail("expected ']]'");
                    p += 2;
                    Value* parent = navigate(path, path.size() - 1);
                    Value* arr = parent->get_mut(path.back());
                    if (!arr) {
                        arr = &parent->insert(path.back(), Value::make(Value::Array));
                        arr->toml_aot = true;
                    } else if (arr->kind != Value::Array || !arr->toml_aot) {
                        fail("'" + path.back() + "' is not an array of tables");
                    }
                    arr->arr.push_back(Value::make(Value::Table));
                    current = &arr->arr.back();
                    current->toml_defined = true;
                } else {
                    if (cur() != ']') fail("expected ']'");
                    ++p;
                    Value* parent = navigate(path, path.size() - 1);
                    Value* tb = parent->get_mut(path.back());
                    if (!tb) {
                        tb = &parent->insert(path.back(), Value::make(Value::Table));
                    } else if (tb->kind != Value::Table || tb->toml_inline) {
                        fail("'" + path.back() + "' is not a table");
                    } else if (tb->toml_defined) {
                        fail("table '" + path.back() + "' defined twice");
                    }
                    tb->toml_defined = true;
                    current = tb;
                }
                end_of_line();
                continue;
            }
            std::vector<std::string> key = dotted_key();
            skip_inline_ws();
            if (cur() != '=') fail("expected '='");
            ++p;
            Value v = value(0);
            assign(*current, key, std::move(v));
            end_of_line();
        }
    }
};

}  // namespace

Value parse_toml(const std::string& text) {
    TomlReader r(text);
    r.parse();
    return std::move(r.root);
}

}  // namespace nrt
