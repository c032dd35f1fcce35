// json_lite.h — the subset of JSON the reference's scene files use, parsed the way the
// reference's nlohmann::json 3.11.3 presents it to scene.cpp:
//   * objects iterate in sorted key order (nlohmann's object_t is a std::map) — this is what
//     makes material ids alphabetical (scene.cpp:53, 131);
//   * numbers keep int/float distinction and convert with static_cast like get<T>().
#pragma once

#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ptj {

struct Value {
    enum Kind { Null, Bool, Int, Float, String, Array, Object } kind = Null;
    bool b = false;
    int64_t i = 0;
    double f = 0.0;
    std::string s;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;

    bool is_number() const { return kind == Int || kind == Float; }
    bool contains(const std::string& k) const { return kind == Object && obj.count(k) != 0; }
    const Value& operator[](const std::string& k) const {
        if (kind != Object) throw std::runtime_error("json: not an object (key " + k + ")");
        auto it = obj.find(k);
        if (it == obj.end()) throw std::runtime_error("json: missing key " + k);
        return it->second;
    }
    const Value& operator[](size_t idx) const {
        if (kind != Array || idx >= arr.size()) throw std::runtime_error("json: bad array index");
        return arr[idx];
    }
    float as_float() const {
        if (kind == Int) return static_cast<float>(i);
        if (kind == Float) return static_cast<float>(f);
        throw std::runtime_error("json: not a number");
    }
    int as_int() const {
        if (kind == Int) return static_cast<int>(i);
        // static_cast like get<int>(); a value outside int (or NaN) has no defined conversion
        if (kind == Float && f > -2147483649.0 && f < 2147483648.0) return static_cast<int>(f);
        if (kind == Float) throw std::runtime_error("json: number out of int range");
        throw std::runtime_error("json: not a number");
    }
    // iteration as nlohmann presents it to scene.cpp: `for (auto& p : objectsData)` over a non-array
    // and `item.key()` over a non-object throw type_error there
    const std::vector<Value>& as_array() const {
        if (kind != Array) throw std::runtime_error("json: not an array");
        return arr;
    }
    const std::map<std::string, Value>& as_object() const {
        if (kind != Object) throw std::runtime_error("json: not an object");
        return obj;
    }
    const std::string& as_string() const {
        if (kind != String) throw std::runtime_error("json: not a string");
        return s;
    }
};

class Parser {
public:
    explicit Parser(const std::string& text) : t_(text) {}
    Value parse() {
        Value v = value();
        ws();
        if (p_ != t_.size()) err("trailing characters");
        return v;
    }

private:
    const std::string& t_;
    size_t p_ = 0;
    int depth_ = 0;   // nesting of arrays / objects (recursive descent: bounded, not the C++ stack)
    static constexpr int kMaxDepth = 256;

    [[noreturn]] void err(const char* m) { throw std::runtime_error(std::string("json: ") + m + " at offset " + std::to_string(p_)); }
    void ws() {
        while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\t' || t_[p_] == '\n' || t_[p_] == '\r')) ++p_;
    }
    char peek() { ws(); return p_ < t_.size() ? t_[p_] : '\0'; }
    void expect(char c) {
        if (peek() != c) err("unexpected character");
        ++p_;
    }
    Value value() {
        char c = peek();
        if (c == '{' || c == '[') {
            if (++depth_ > kMaxDepth) err("nesting too deep");
            Value v = c == '{' ? object() : array();
            --depth_;
            return v;
        }
        if (c == '"') { Value v; v.kind = Value::String; v.s = str(); return v; }
        if (c == 't' || c == 'f' || c == 'n') return literal();
        return number();
    }
    Value object() {
        Value v;
        v.kind = Value::Object;
        expect('{');
        if (peek() == '}') { ++p_; return v; }
        for (;;) {
            if (peek() != '"') err("expected key");
            std::string k = str();
            expect(':');
            v.obj[k] = value();   // duplicate keys: last one wins
            char c = peek();
            ++p_;
            if (c == '}') break;
            if (c != ',') err("expected , or }");
        }
        return v;
    }
    Value array() {
        Value v;
        v.kind = Value::Array;
        expect('[');
        if (peek() == ']') { ++p_; return v; }
        for (;;) {
            v.arr.push_back(value());
            char c = peek();
            ++p_;
            if (c == ']') break;
            if (c != ',') err("expected , or ]");
        }
        return v;
    }
    std::string str() {
        expect('"');
        std::string out;
        while (p_ < t_.size() && t_[p_] != '"') {
            char c = t_[p_++];
            if (c == '\\') {
                if (p_ >= t_.size()) err("bad escape");
                char e = t_[p_++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (p_ + 4 > t_.size()) err("bad \\u");
                        unsigned cp = (unsigned)std::strtoul(t_.substr(p_, 4).c_str(), nullptr, 16);
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
        if (p_ >= t_.size()) err("unterminated string");
        ++p_;
        return out;
    }
    Value literal() {
        Value v;
        if (t_.compare(p_, 4, "true") == 0) { v.kind = Value::Bool; v.b = true; p_ += 4; }
        else if (t_.compare(p_, 5, "false") == 0) { v.kind = Value::Bool; v.b = false; p_ += 5; }
        else if (t_.compare(p_, 4, "null") == 0) { v.kind = Value::Null; p_ += 4; }
        else err("bad literal");
        return v;
    }
    Value number() {
        size_t start = p_;
        bool is_float = false;
        if (t_[p_] == '-' || t_[p_] == '+') ++p_;
        while (p_ < t_.size()) {
            char c = t_[p_];
            if (c >= '0' && c <= '9') { ++p_; continue; }
            if (c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-') { is_float = true; ++p_; continue; }
            break;
        }
        if (p_ == start) err("bad value");
        std::string tok = t_.substr(start, p_ - start);
        Value v;
        if (is_float) { v.kind = Value::Float; v.f = std::strtod(tok.c_str(), nullptr); }
        else { v.kind = Value::Int; v.i = std::strtoll(tok.c_str(), nullptr, 10); }
        return v;
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace ptj
