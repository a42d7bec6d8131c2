// Minimal JSON reader for the namespace AST (internal/schema/.snapshots format).
// Objects keep key order (relation order matters for ASTRelationFor's first match,
// internal/namespace/definitions.go:56-60).
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace keto::json {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0;
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;

    const Value *get(const std::string &k) const {
        if (kind != Object) return nullptr;
        for (auto &kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    bool has(const std::string &k) const { return get(k) != nullptr; }
};

class Parser {
  public:
    explicit Parser(const std::string &s) : s_(s) {}
    Value parse() {
        Value v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

  private:
    const std::string &s_;
    size_t i_ = 0;

    [[noreturn]] void fail(const char *what) {
        throw std::runtime_error(std::string("namespace JSON: ") + what + " at offset " + std::to_string(i_));
    }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r')) i_++;
    }
    char peek() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        return s_[i_];
    }
    void expect(char c) {
        if (peek() != c) fail("unexpected character");
        i_++;
    }
    bool lit(const char *w) {
        size_t n = std::char_traits<char>::length(w);
        if (s_.compare(i_, n, w) == 0) {
            i_ += n;
            return true;
        }
        return false;
    }
    static void put_utf8(std::string &o, uint32_t cp) {
        if (cp < 0x80) o += char(cp);
        else if (cp < 0x800) {
            o += char(0xC0 | (cp >> 6));
            o += char(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
            o += char(0xE0 | (cp >> 12));
            o += char(0x80 | ((cp >> 6) & 0x3F));
            o += char(0x80 | (cp & 0x3F));
        } else {
            o += char(0xF0 | (cp >> 18));
            o += char(0x80 | ((cp >> 12) & 0x3F));
            o += char(0x80 | ((cp >> 6) & 0x3F));
            o += char(0x80 | (cp & 0x3F));
        }
    }
    uint32_t hex4() {
        if (i_ + 4 > s_.size()) fail("bad \\u escape");
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) {
            char c = s_[i_++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else fail("bad hex digit");
        }
        return v;
    }
    std::string string() {
        expect('"');
        std::string o;
        while (true) {
            if (i_ >= s_.size()) fail("unterminated string");
            char c = s_[i_++];
            if (c == '"') break;
            if (c != '\\') {
                o += c;
                continue;
            }
            if (i_ >= s_.size()) fail("bad escape");
            char e = s_[i_++];
            switch (e) {
            case '"': o += '"'; break;
            case '\\': o += '\\'; break;
            case '/': o += '/'; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case 'n': o += '\n'; break;
            case 'r': o += '\r'; break;
            case 't': o += '\t'; break;
            case 'u': {
                uint32_t cp = hex4();
                if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
                    i_ += 2;
                    uint32_t lo = hex4();
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                }
                put_utf8(o, cp);
                break;
            }
            default: fail("bad escape");
            }
        }
        return o;
    }
    Value value() {
        Value v;
        char c = peek();
        if (c == '{') {
            i_++;
            v.kind = Value::Object;
            if (peek() == '}') {
                i_++;
                return v;
            }
            while (true) {
                std::string k = string();
                expect(':');
                v.obj.emplace_back(std::move(k), value());
                if (peek() == ',') {
                    i_++;
                    continue;
                }
                expect('}');
                return v;
            }
        }
        if (c == '[') {
            i_++;
            v.kind = Value::Array;
            if (peek() == ']') {
                i_++;
                return v;
            }
            while (true) {
                v.arr.push_back(value());
                if (peek() == ',') {
                    i_++;
                    continue;
                }
                expect(']');
                return v;
            }
        }
        if (c == '"') {
            v.kind = Value::String;
            v.str = string();
            return v;
        }
        if (lit("true")) {
            v.kind = Value::Bool;
            v.b = true;
            return v;
        }
        if (lit("false")) {
            v.kind = Value::Bool;
            return v;
        }
        if (lit("null")) return v;
        size_t st = i_;
        while (i_ < s_.size() && (isdigit((unsigned char)s_[i_]) || s_[i_] == '-' || s_[i_] == '+' ||
                                  s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E'))
            i_++;
        if (st == i_) fail("unexpected token");
        v.kind = Value::Number;
        v.num = std::stod(s_.substr(st, i_ - st));
        return v;
    }
};

inline Value parse(const std::string &s) { return Parser(s).parse(); }

}  // namespace keto::json
