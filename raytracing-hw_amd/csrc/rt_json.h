// rt_json.h — minimal JSON reader for glTF 2.0 documents (host only).
//
// The reference parses glTF with tinygltf v2.8.10 on nlohmann::json
// (thirdparty/tinygltf/tiny_gltf.h); only the handful of fields scene_parser.cpp reads are
// needed here.  Numbers are kept as double via strtod (correctly rounded, like nlohmann's
// number parser), so every value reaches the (float) casts of scene_parser.cpp unchanged.
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rtj {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;

    bool is_null() const { return kind == Null; }
    bool has(const std::string &k) const { return kind == Object && obj.count(k) != 0; }
    const Value &operator[](const std::string &k) const {
        static const Value null_value;
        if (kind != Object) return null_value;
        auto it = obj.find(k);
        return it == obj.end() ? null_value : it->second;
    }
    const Value &operator[](size_t i) const {
        static const Value null_value;
        return (kind == Array && i < arr.size()) ? arr[i] : null_value;
    }
    size_t size() const { return kind == Array ? arr.size() : (kind == Object ? obj.size() : 0); }
    double number(double dflt) const { return kind == Number ? num : dflt; }
    int integer(int dflt) const { return kind == Number ? (int)num : dflt; }
    std::vector<double> numbers() const {
        std::vector<double> v;
        if (kind == Array)
            for (auto &e : arr) v.push_back(e.num);
        return v;
    }
};

class Parser {
public:
    explicit Parser(const std::string &text) : s_(text) {}
    Value parse() {
        Value v = value();
        ws();
        if (p_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string &s_;
    size_t p_ = 0;

    [[noreturn]] void fail(const char *what) {
        throw std::runtime_error(std::string("[json] ") + what + " at offset " + std::to_string(p_));
    }
    void ws() {
        while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\n' || s_[p_] == '\r' || s_[p_] == '\t')) ++p_;
    }
    bool lit(const char *w) {
        size_t n = std::char_traits<char>::length(w);
        if (s_.compare(p_, n, w) == 0) { p_ += n; return true; }
        return false;
    }
    Value value() {
        ws();
        if (p_ >= s_.size()) fail("unexpected end");
        Value v;
        char c = s_[p_];
        if (c == '{') {
            v.kind = Value::Object;
            ++p_;
            ws();
            if (p_ < s_.size() && s_[p_] == '}') { ++p_; return v; }
            for (;;) {
                ws();
                if (p_ >= s_.size() || s_[p_] != '"') fail("expected key");
                std::string k = string();
                ws();
                if (p_ >= s_.size() || s_[p_] != ':') fail("expected ':'");
                ++p_;
                v.obj[k] = value();
                ws();
                if (p_ < s_.size() && s_[p_] == ',') { ++p_; continue; }
                if (p_ < s_.size() && s_[p_] == '}') { ++p_; return v; }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = Value::Array;
            ++p_;
            ws();
            if (p_ < s_.size() && s_[p_] == ']') { ++p_; return v; }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (p_ < s_.size() && s_[p_] == ',') { ++p_; continue; }
                if (p_ < s_.size() && s_[p_] == ']') { ++p_; return v; }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') { v.kind = Value::String; v.str = string(); return v; }
        if (lit("true")) { v.kind = Value::Bool; v.b = true; return v; }
        if (lit("false")) { v.kind = Value::Bool; v.b = false; return v; }
        if (lit("null")) return v;
        const char *begin = s_.c_str() + p_;
        char *end = nullptr;
        v.num = std::strtod(begin, &end);
        if (end == begin) fail("bad value");
        v.kind = Value::Number;
        p_ += (size_t)(end - begin);
        return v;
    }
    std::string string() {
        std::string out;
        ++p_;  // opening quote
        while (p_ < s_.size() && s_[p_] != '"') {
            char c = s_[p_++];
            if (c == '\\') {
                if (p_ >= s_.size()) fail("bad escape");
                char e = s_[p_++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (p_ + 4 > s_.size()) fail("bad \\u escape");
                        unsigned cp = (unsigned)std::strtoul(s_.substr(p_, 4).c_str(), nullptr, 16);
                        p_ += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (p_ >= s_.size()) fail("unterminated string");
        ++p_;
        return out;
    }
};

inline Value parse(const std::string &text) { return Parser(text).parse(); }

}  // namespace rtj
