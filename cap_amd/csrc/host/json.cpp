// json.cpp -- see json.hpp.  A single-pass recursive-descent reader: syntax
// errors abort the parse (Go runs checkValid over the whole text before it
// decodes anything, so a syntax error anywhere rejects the document).
#include "json.hpp"

#include "hostmem.hpp"

#include <algorithm>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

namespace capjwt {
namespace json {

// ---------------------------------------------------------------- arenas
namespace {
thread_local Arena* tl_arena = nullptr;
}  // namespace

Arena* current_arena() { return tl_arena; }
ArenaScope::ArenaScope(Arena* a) : prev_(tl_arena) { tl_arena = a; }
ArenaScope::~ArenaScope() { tl_arena = prev_; }

Arena::~Arena() {
  for (void* b : blocks_) hostmem::block_put(b);
  for (void* b : big_) ::operator delete(b);
}

void Str::assign_in(Arena* a, const char* p, size_t n) {
  if (n > 0xFFFFFFF0u) throw std::bad_alloc();
  if (n <= kInline) {
    char tmp[kInline + 1];
    std::memcpy(tmp, p, n);                        // p may point into this string
    release();
    std::memcpy(s_, tmp, n);
    s_[n] = 0;
    n_ = (uint32_t)n;
    return;
  }
  char* q = static_cast<char*>(a ? a->alloc(n + 1) : ::operator new(n + 1));
  std::memcpy(q, p, n);
  q[n] = 0;
  release();
  p_ = q;
  n_ = (uint32_t)n;
  arena_ = a != nullptr;
}

void Str::take(Str& o) {
  if (o.n_ <= kInline) {
    std::memcpy(s_, o.s_, o.n_ + 1);
    n_ = o.n_;
  } else if (o.arena_ && !current_arena()) {       // leaving the batch: to the heap
    assign_in(nullptr, o.p_, o.n_);
  } else {
    p_ = o.p_;
    n_ = o.n_;
    arena_ = o.arena_;
    o.n_ = 0;
    o.arena_ = false;
  }
  o.release();
}

void* Arena::alloc(size_t bytes) {
  bytes = (bytes + 15) & ~size_t(15);
  used_ += bytes;
  if (bytes > hostmem::kBlock / 4) {               // a huge object: its own allocation
    big_.push_back(::operator new(bytes));
    return big_.back();
  }
  if (bytes > left_) {
    blocks_.push_back(hostmem::block_get());
    cur_ = static_cast<char*>(blocks_.back());
    left_ = hostmem::kBlock;
  }
  void* r = cur_;
  cur_ += bytes;
  left_ -= bytes;
  return r;
}

const Value* Value::get(std::string_view key) const {
  if (kind != Object) return nullptr;
  for (const auto& m : obj)
    if (m.first == key) return &m.second;
  return nullptr;
}

void put_utf8(std::string& o, uint32_t r) {
  if (r < 0x80) {
    o.push_back((char)r);
  } else if (r < 0x800) {
    o.push_back((char)(0xC0 | (r >> 6)));
    o.push_back((char)(0x80 | (r & 0x3F)));
  } else if (r < 0x10000) {
    o.push_back((char)(0xE0 | (r >> 12)));
    o.push_back((char)(0x80 | ((r >> 6) & 0x3F)));
    o.push_back((char)(0x80 | (r & 0x3F)));
  } else {
    o.push_back((char)(0xF0 | (r >> 18)));
    o.push_back((char)(0x80 | ((r >> 12) & 0x3F)));
    o.push_back((char)(0x80 | ((r >> 6) & 0x3F)));
    o.push_back((char)(0x80 | (r & 0x3F)));
  }
}

// Decode one UTF-8 sequence at s[i..n) the way Go's utf8.DecodeRune does:
// returns the rune and its width, or (0xFFFD, 1) for any invalid encoding.
uint32_t decode_rune(const unsigned char* s, size_t n, size_t* w) {
  const unsigned c = s[0];
  *w = 1;
  if (c < 0x80) return c;
  auto cont = [&](size_t k) { return k < n && (s[k] & 0xC0) == 0x80; };
  if (c >= 0xC2 && c <= 0xDF) {
    if (!cont(1)) return 0xFFFD;
    *w = 2;
    return ((c & 0x1F) << 6) | (s[1] & 0x3F);
  }
  if (c >= 0xE0 && c <= 0xEF) {
    if (n < 2) return 0xFFFD;
    const unsigned lo = c == 0xE0 ? 0xA0 : 0x80, hi = c == 0xED ? 0x9F : 0xBF;
    if (s[1] < lo || s[1] > hi || !cont(2)) return 0xFFFD;
    *w = 3;
    return ((c & 0x0F) << 12) | ((s[1] & 0x3F) << 6) | (s[2] & 0x3F);
  }
  if (c >= 0xF0 && c <= 0xF4) {
    if (n < 2) return 0xFFFD;
    const unsigned lo = c == 0xF0 ? 0x90 : 0x80, hi = c == 0xF4 ? 0x8F : 0xBF;
    if (s[1] < lo || s[1] > hi || !cont(2) || !cont(3)) return 0xFFFD;
    *w = 4;
    return ((c & 0x07) << 18) | ((s[1] & 0x3F) << 12) | ((s[2] & 0x3F) << 6) | (s[3] & 0x3F);
  }
  return 0xFFFD;
}

namespace {
constexpr int kMaxDepth = 10000;   // encoding/json scanner maxNestingDepth


struct Reader {
  const unsigned char* p;
  const unsigned char* end;
  const unsigned char* begin;
  std::string err;
  Arena* arena = nullptr;          // the tree's containers and texts go here (parse under an ArenaScope)

  bool fail(const char* what) {
    if (err.empty()) {
      if (p >= end) {
        err = "unexpected end of JSON input";
      } else {
        char ch[8];
        if (*p >= 0x20 && *p < 0x7F) snprintf(ch, sizeof(ch), "'%c'", (char)*p);
        else snprintf(ch, sizeof(ch), "'\\x%02x'", (unsigned)*p);
        err = std::string("invalid character ") + ch + " " + what;
      }
    }
    return false;
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static int hex(unsigned c) {
    if (c >= '0' && c <= '9') return (int)(c - '0');
    if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
    return -1;
  }
  bool u4(uint32_t* r) {
    if (end - p < 4) { p = end; return fail(""); }
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      const int h = hex(p[i]);
      if (h < 0) { p += i; return fail("in \\u hexadecimal character escape"); }
      v = v << 4 | (uint32_t)h;
    }
    p += 4;
    *r = v;
    return true;
  }

  bool string(Str* out) {
    // at the opening quote
    ++p;
    const unsigned char* run = p;
    // fast scan: plain ASCII without escapes
    while (p < end && *p != '"' && *p != '\\' && *p >= 0x20 && *p < 0x80) ++p;
    if (p < end && *p == '"') {
      out->assign_in(arena, (const char*)run, (size_t)(p - run));
      ++p;
      return true;
    }
    thread_local std::string scratch;
    if (!string_slow(&scratch, run)) return false;
    out->assign_in(arena, scratch.data(), scratch.size());
    return true;
  }

  bool string(std::string* out) {
    ++p;
    const unsigned char* run = p;
    while (p < end && *p != '"' && *p != '\\' && *p >= 0x20 && *p < 0x80) ++p;
    if (p < end && *p == '"') {
      out->assign((const char*)run, (size_t)(p - run));
      ++p;
      return true;
    }
    return string_slow(out, run);
  }

  // the rest of a string with escapes or non-ASCII bytes: p is past the plain
  // prefix that starts at `run`
  bool string_slow(std::string* out, const unsigned char* run) {
    out->assign((const char*)run, (size_t)(p - run));
    while (true) {
      if (p >= end) return fail("");
      const unsigned c = *p;
      if (c == '"') { ++p; return true; }
      if (c < 0x20) return fail("in string literal");
      if (c == '\\') {
        ++p;
        if (p >= end) return fail("");
        const unsigned e = *p++;
        switch (e) {
          case '"': out->push_back('"'); break;
          case '\\': out->push_back('\\'); break;
          case '/': out->push_back('/'); break;
          case 'b': out->push_back('\b'); break;
          case 'f': out->push_back('\f'); break;
          case 'n': out->push_back('\n'); break;
          case 'r': out->push_back('\r'); break;
          case 't': out->push_back('\t'); break;
          case 'u': {
            uint32_t r = 0;
            if (!u4(&r)) return false;
            if (r >= 0xD800 && r < 0xE000) {
              // utf16 surrogate: valid only as a high+low pair written as two escapes
              uint32_t r2 = 0;
              if (r < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                const unsigned char* save = p;
                p += 2;
                bool ok = true;
                uint32_t v = 0;
                for (int i = 0; i < 4; ++i) {
                  const int h = hex(p[i]);
                  if (h < 0) { ok = false; break; }
                  v = v << 4 | (uint32_t)h;
                }
                if (ok && v >= 0xDC00 && v < 0xE000) {
                  p += 4;
                  r2 = v;
                  put_utf8(*out, 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00));
                  break;
                }
                p = save;          // the next escape is decoded on its own
              }
              put_utf8(*out, 0xFFFD);
            } else {
              put_utf8(*out, r);
            }
            break;
          }
          default:
            --p;
            return fail("in string escape code");
        }
        continue;
      }
      if (c < 0x80) { out->push_back((char)c); ++p; continue; }
      size_t w;
      const uint32_t r = decode_rune(p, (size_t)(end - p), &w);
      if (r == 0xFFFD && w == 1) put_utf8(*out, 0xFFFD);
      else out->append((const char*)p, w);
      p += w;
    }
  }

  bool number(Value* v) {
    const unsigned char* s = p;
    const bool neg = *p == '-';
    if (neg) ++p;
    if (p >= end) return fail("in numeric literal");
    uint64_t iv = 0;
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') iv = iv * 10 + (uint64_t)(*p++ - '0');
    } else {
      return fail("in numeric literal");
    }
    const size_t ndig = (size_t)(p - s) - neg;
    if (ndig <= 15 && (p >= end || (*p != '.' && *p != 'e' && *p != 'E'))) {
      // an integer below 10^15 is exact in float64: ParseFloat's result without strtod
      v->kind = Value::Number;
      v->str.assign_in(arena, (const char*)s, (size_t)(p - s));
      v->num = neg ? -(double)iv : (double)iv;
      v->num_range_err = false;
      return true;
    }
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("after decimal point in numeric literal");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("in exponent of numeric literal");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    v->kind = Value::Number;
    v->str.assign_in(arena, (const char*)s, (size_t)(p - s));
    // strconv.ParseFloat: correctly rounded; overflow -> ErrRange, underflow -> 0
    errno = 0;
    const double d = std::strtod(v->str.c_str(), nullptr);
    v->num = d;
    v->num_range_err = std::isinf(d);
    return true;
  }

  bool literal(const char* word, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      if (p >= end) return fail("");
      if (*p != (unsigned char)word[i]) return fail(i == 0 ? "looking for beginning of value" : "in literal");
      ++p;
    }
    return true;
  }

  bool value(Value* v, int depth) {
    ws();
    if (p >= end) return fail("");
    switch (*p) {
      case '{': return object(v, depth + 1);
      case '[': return array(v, depth + 1);
      case '"': v->kind = Value::String; return string(&v->str);
      case 't': v->kind = Value::Bool; v->b = true; return literal("true", 4);
      case 'f': v->kind = Value::Bool; v->b = false; return literal("false", 5);
      case 'n': v->kind = Value::Null; return literal("null", 4);
      default:
        if (*p == '-' || (*p >= '0' && *p <= '9')) return number(v);
        return fail("looking for beginning of value");
    }
  }

  bool array(Value* v, int depth) {
    if (depth > kMaxDepth) { err = "exceeded max depth"; return false; }
    v->kind = Value::Array;
    ++p;
    ws();
    if (p < end && *p == ']') { ++p; return true; }
    while (true) {
      v->arr.emplace_back();
      if (!value(&v->arr.back(), depth)) return false;
      ws();
      if (p >= end) return fail("");
      if (*p == ',') { ++p; continue; }
      if (*p == ']') { ++p; return true; }
      return fail("after array element");
    }
  }

  bool object(Value* v, int depth) {
    if (depth > kMaxDepth) { err = "exceeded max depth"; return false; }
    v->kind = Value::Object;
    ++p;
    ws();
    if (p < end && *p == '}') { ++p; return true; }
    std::unordered_map<std::string, size_t> index;   // only for large objects
    v->obj.reserve(8);                                // one allocation for a claims set
    while (true) {
      ws();
      if (p >= end) return fail("");
      if (*p != '"') return fail("looking for beginning of object key string");
      // the member is parsed in place at the end of the object; a duplicate
      // name then moves its value onto the earlier member (map assignment:
      // the last duplicate wins)
      v->obj.emplace_back();
      const size_t at_new = v->obj.size() - 1;
      if (!string(&v->obj[at_new].first)) return false;
      ws();
      if (p >= end) return fail("");
      if (*p != ':') return fail("after object key");
      ++p;
      if (!value(&v->obj[at_new].second, depth)) return false;
      const std::string& key = v->obj[at_new].first;
      size_t at = at_new;
      if (at_new < 16) {
        for (size_t i = 0; i < at_new; ++i)
          if (v->obj[i].first == key) { at = i; break; }
        if (at == at_new && at_new == 15)
          for (size_t i = 0; i <= at_new; ++i) index.emplace(v->obj[i].first, i);
      } else {
        auto it = index.find(key);
        if (it != index.end()) at = it->second;
        else index.emplace(key, at_new);
      }
      if (at != at_new) {
        v->obj[at].second = std::move(v->obj[at_new].second);
        v->obj.pop_back();
      }
      ws();
      if (p >= end) return fail("");
      if (*p == ',') { ++p; continue; }
      if (*p == '}') { ++p; return true; }
      return fail("after object key:value pair");
    }
  }
};

void escape_string(std::string& o, std::string_view s) {
  static const char* hexd = "0123456789abcdef";
  o.push_back('"');
  const unsigned char* p = (const unsigned char*)s.data();
  const size_t n = s.size();
  for (size_t i = 0; i < n;) {
    const unsigned c = p[i];
    if (c < 0x80) {
      if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') {
        o.push_back((char)c);
      } else {
        o.push_back('\\');
        switch (c) {
          case '"': o.push_back('"'); break;
          case '\\': o.push_back('\\'); break;
          case '\b': o.push_back('b'); break;
          case '\f': o.push_back('f'); break;
          case '\n': o.push_back('n'); break;
          case '\r': o.push_back('r'); break;
          case '\t': o.push_back('t'); break;
          default:
            o += "u00";
            o.push_back(hexd[c >> 4]);
            o.push_back(hexd[c & 15]);
        }
      }
      ++i;
      continue;
    }
    size_t w;
    const uint32_t r = decode_rune(p + i, n - i, &w);
    if (r == 0xFFFD && w == 1) {
      o += "\\ufffd";
    } else if (r == 0x2028 || r == 0x2029) {
      o += r == 0x2028 ? "\\u2028" : "\\u2029";
    } else {
      o.append((const char*)p + i, w);
    }
    i += w;
  }
  o.push_back('"');
}

void marshal_into(std::string& o, const Value& v) {
  switch (v.kind) {
    case Value::Null: o += "null"; break;
    case Value::Bool: o += v.b ? "true" : "false"; break;
    case Value::Number: o += format_float(v.num); break;
    case Value::String: escape_string(o, v.str); break;
    case Value::Array:
      o.push_back('[');
      for (size_t i = 0; i < v.arr.size(); ++i) {
        if (i) o.push_back(',');
        marshal_into(o, v.arr[i]);
      }
      o.push_back(']');
      break;
    case Value::Object: {
      std::vector<const Member*> ms;
      ms.reserve(v.obj.size());
      for (const auto& m : v.obj) ms.push_back(&m);
      std::sort(ms.begin(), ms.end(), [](const Member* a, const Member* b) { return a->first < b->first; });
      o.push_back('{');
      for (size_t i = 0; i < ms.size(); ++i) {
        if (i) o.push_back(',');
        escape_string(o, ms[i]->first);
        o.push_back(':');
        marshal_into(o, ms[i]->second);
      }
      o.push_back('}');
      break;
    }
  }
}

}  // namespace

bool parse(std::string_view text, Value* out, std::string* err) {
  Reader r;
  r.arena = current_arena();
  r.begin = r.p = (const unsigned char*)text.data();
  r.end = r.p + text.size();
  *out = Value();
  if (!r.value(out, 0)) {
    if (err) *err = r.err.empty() ? "invalid JSON" : r.err;
    return false;
  }
  r.ws();
  if (r.p != r.end) {
    r.fail("after top-level value");
    if (err) *err = r.err;
    return false;
  }
  return true;
}

bool has_range_error(const Value& v) {
  switch (v.kind) {
    case Value::Number: return v.num_range_err;
    case Value::Array:
      for (const auto& e : v.arr)
        if (has_range_error(e)) return true;
      return false;
    case Value::Object:
      for (const auto& m : v.obj)
        if (has_range_error(m.second)) return true;
      return false;
    default: return false;
  }
}

std::string format_float(double f) {
  char buf[64];
  const double a = std::fabs(f);
  const bool sci = a != 0 && (a < 1e-6 || a >= 1e21);
  auto r = std::to_chars(buf, buf + sizeof(buf), f, sci ? std::chars_format::scientific : std::chars_format::fixed);
  std::string s(buf, r.ptr);
  if (sci) {
    const size_t n = s.size();
    if (n >= 4 && s[n - 4] == 'e' && s[n - 3] == '-' && s[n - 2] == '0') s.erase(n - 2, 1);
  }
  return s;
}

std::string marshal(const Value& v) {
  std::string o;
  marshal_into(o, v);
  return o;
}

}  // namespace json
}  // namespace capjwt
