// vf_json.h -- the small JSON reader and writer the native control plane needs for wire v1 / v2
// message heads (vfilter/wire.py): requests {"credit", "shm", "wid", "numa", "wire"}, v1 frame
// lists and columns, v2 result heads {"pid", "wid", "start", "end", "errors", ...}.  A strict
// recursive-descent parser over a bounded buffer (depth <= 64, no trailing garbage), numbers kept
// as double plus an exact int64 when integral.  Heads are at most a few KB per batch.
#pragma once

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace vfjson {

struct Value {
    enum Type { Null, Bool, Num, Str, Arr, Obj } type = Null;
    bool b = false;
    double num = 0.0;
    int64_t i = 0;
    bool is_int = false;
    std::string s;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;

    const Value* get(const char* key) const {
        if (type != Obj) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    bool null() const { return type == Null; }
    int64_t as_int(int64_t dflt = 0) const {
        if (type == Num) return is_int ? i : (int64_t)num;
        if (type == Bool) return b ? 1 : 0;
        return dflt;
    }
    double as_num(double dflt = 0.0) const { return type == Num ? num : dflt; }
};

class Parser {
  public:
    Parser(const char* p, size_t n) : p_(p), end_(p + n) {}
    bool parse(Value& out) {
        ws();
        if (!value(out, 0)) return false;
        ws();
        return p_ == end_;
    }

  private:
    const char* p_;
    const char* end_;

    void ws() {
        while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool lit(const char* w) {
        size_t n = std::strlen(w);
        if ((size_t)(end_ - p_) < n || std::memcmp(p_, w, n) != 0) return false;
        p_ += n;
        return true;
    }
    bool value(Value& v, int depth) {
        if (depth > 64 || p_ >= end_) return false;
        switch (*p_) {
            case 'n': v.type = Value::Null; return lit("null");
            case 't': v.type = Value::Bool; v.b = true; return lit("true");
            case 'f': v.type = Value::Bool; v.b = false; return lit("false");
            case '"': v.type = Value::Str; return str(v.s);
            case '[': {
                v.type = Value::Arr;
                ++p_;
                ws();
                if (p_ < end_ && *p_ == ']') { ++p_; return true; }
                for (;;) {
                    v.arr.emplace_back();
                    ws();
                    if (!value(v.arr.back(), depth + 1)) return false;
                    ws();
                    if (p_ >= end_) return false;
                    if (*p_ == ',') { ++p_; continue; }
                    if (*p_ == ']') { ++p_; return true; }
                    return false;
                }
            }
            case '{': {
                v.type = Value::Obj;
                ++p_;
                ws();
                if (p_ < end_ && *p_ == '}') { ++p_; return true; }
                for (;;) {
                    ws();
                    std::string k;
                    if (p_ >= end_ || *p_ != '"' || !str(k)) return false;
                    ws();
                    if (p_ >= end_ || *p_ != ':') return false;
                    ++p_;
                    ws();
                    v.obj.emplace_back(std::move(k), Value());
                    if (!value(v.obj.back().second, depth + 1)) return false;
                    ws();
                    if (p_ >= end_) return false;
                    if (*p_ == ',') { ++p_; continue; }
                    if (*p_ == '}') { ++p_; return true; }
                    return false;
                }
            }
            default: return number(v);
        }
    }
    static void utf8(std::string& o, uint32_t c) {
        if (c < 0x80) {
            o += (char)c;
        } else if (c < 0x800) {
            o += (char)(0xC0 | (c >> 6));
            o += (char)(0x80 | (c & 0x3F));
        } else if (c < 0x10000) {
            o += (char)(0xE0 | (c >> 12));
            o += (char)(0x80 | ((c >> 6) & 0x3F));
            o += (char)(0x80 | (c & 0x3F));
        } else {
            o += (char)(0xF0 | (c >> 18));
            o += (char)(0x80 | ((c >> 12) & 0x3F));
            o += (char)(0x80 | ((c >> 6) & 0x3F));
            o += (char)(0x80 | (c & 0x3F));
        }
    }
    bool hex4(uint32_t& c) {
        if (end_ - p_ < 4) return false;
        c = 0;
        for (int k = 0; k < 4; ++k) {
            char h = *p_++;
            c <<= 4;
            if (h >= '0' && h <= '9') c |= (uint32_t)(h - '0');
            else if (h >= 'a' && h <= 'f') c |= (uint32_t)(h - 'a' + 10);
            else if (h >= 'A' && h <= 'F') c |= (uint32_t)(h - 'A' + 10);
            else return false;
        }
        return true;
    }
    bool str(std::string& o) {
        ++p_;  // opening quote
        while (p_ < end_) {
            char c = *p_++;
            if (c == '"') return true;
            if ((unsigned char)c < 0x20) return false;
            if (c != '\\') { o += c; continue; }
            if (p_ >= end_) return false;
            char e = *p_++;
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
                    uint32_t cp;
                    if (!hex4(cp)) return false;
                    if (cp >= 0xD800 && cp < 0xDC00) {  // surrogate pair
                        uint32_t lo;
                        if (end_ - p_ < 6 || p_[0] != '\\' || p_[1] != 'u') return false;
                        p_ += 2;
                        if (!hex4(lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(o, cp);
                    break;
                }
                default: return false;
            }
        }
        return false;
    }
    bool number(Value& v) {
        const char* s = p_;
        bool integral = true;
        if (p_ < end_ && *p_ == '-') ++p_;
        if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) return false;
        while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        if (p_ < end_ && *p_ == '.') {
            integral = false;
            ++p_;
            if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) return false;
            while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        if (p_ < end_ && (*p_ == 'e' || *p_ == 'E')) {
            integral = false;
            ++p_;
            if (p_ < end_ && (*p_ == '+' || *p_ == '-')) ++p_;
            if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) return false;
            while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        std::string t(s, p_);
        v.type = Value::Num;
        v.num = std::strtod(t.c_str(), nullptr);
        if (integral && t.size() < 19) {
            v.i = std::strtoll(t.c_str(), nullptr, 10);
            v.is_int = true;
        } else if (integral) {  // beyond 18 digits: exact only if it fits
            errno = 0;
            long long x = std::strtoll(t.c_str(), nullptr, 10);
            v.is_int = errno == 0;
            v.i = x;
        } else if (std::isfinite(v.num) && v.num == std::floor(v.num) && std::fabs(v.num) < 9.0e15) {
            v.i = (int64_t)v.num;
            v.is_int = true;
        }
        return true;
    }
};

inline bool parse(const void* p, size_t n, Value& out) {
    Parser ps((const char*)p, n);
    return ps.parse(out);
}

// writer helpers
inline void put_str(std::string& o, const std::string& s) {
    o += '"';
    for (unsigned char c : s) {
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            default:
                if (c < 0x20) {
                    char b[8];
                    std::snprintf(b, sizeof b, "\\u%04x", c);
                    o += b;
                } else {
                    o += (char)c;
                }
        }
    }
    o += '"';
}

inline void put_int(std::string& o, int64_t v) {
    char b[24];
    int n = std::snprintf(b, sizeof b, "%lld", (long long)v);
    o.append(b, (size_t)n);
}

inline void put_num(std::string& o, double v) {
    char b[32];
    int n = std::snprintf(b, sizeof b, "%.17g", v);
    o.append(b, (size_t)n);
}

}  // namespace vfjson
