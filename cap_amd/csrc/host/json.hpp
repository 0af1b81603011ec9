// json.hpp -- a JSON reader with Go encoding/json semantics, for the host side
// of the verifier (header decode, payload -> claims map, JWKS documents).
//
// Semantics restated from Go's encoding/json (and go-jose v2.5.1's fork of it,
// which behaves identically for the values read here); SURVEY.md Appendix A:
//   * full syntax check before any value is used (RFC 8259 grammar, no
//     trailing garbage, nesting depth <= 10000 as Go's scanner enforces);
//   * objects: duplicate member names -> the last one wins (map assignment);
//   * strings: escapes decoded; invalid UTF-8 and lone surrogates become
//     U+FFFD (decode.go unquote), never an error;
//   * numbers into interface{} are float64: a literal that overflows float64
//     is an UnmarshalTypeError (strconv.ParseFloat ErrRange); underflow is 0.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <string_view>
#include <type_traits>
#include <utility>
#include <vector>

namespace capjwt {
namespace json {

// ---------------------------------------------------------------- batch arenas
// A bump allocator for the containers of the claims trees of one batch
// (hostmem.hpp explains why).  Its blocks come from the hostmem pool and go
// back to it when the arena dies; nothing allocated in it is freed one by one.
class Arena {
 public:
  Arena() = default;
  ~Arena();
  Arena(const Arena&) = delete;
  Arena& operator=(const Arena&) = delete;
  void* alloc(size_t bytes);              // 16-byte aligned
  size_t used() const { return used_; }
 private:
  std::vector<void*> blocks_, big_;       // pooled blocks; oversized requests (malloc)
  char* cur_ = nullptr;
  size_t left_ = 0, used_ = 0;
};

// While an ArenaScope is alive, containers that grow on this thread take their
// storage from its arena.  Scopes only exist inside the batch passes of the
// host layer, around trees whose owner (the batch's Results) keeps the arena.
class ArenaScope {
 public:
  explicit ArenaScope(Arena* a);
  ~ArenaScope();
  ArenaScope(const ArenaScope&) = delete;
  ArenaScope& operator=(const ArenaScope&) = delete;
 private:
  Arena* prev_;
};
Arena* current_arena();

// The array / object storage of a Value: a vector that allocates from the
// current arena when one is in scope (else from the heap) and never frees
// arena storage.  A move OUT of arena storage with no arena in scope -- a
// claims map leaving its batch, e.g. Validator::Validate's one result --
// deep-moves the elements to the heap, so a tree never outlives its arena.
template <class T>
class Vec {
 public:
  Vec() = default;
  ~Vec() { destroy(); }
  Vec(const Vec& o) { copy_from(o); }
  Vec(Vec&& o) noexcept { take(o); }
  Vec& operator=(const Vec& o) {
    if (this != &o) { destroy(); copy_from(o); }
    return *this;
  }
  Vec& operator=(Vec&& o) noexcept {
    if (this != &o) { destroy(); take(o); }
    return *this;
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T* begin() { return p_; }
  T* end() { return p_ + n_; }
  const T* begin() const { return p_; }
  const T* end() const { return p_ + n_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  T& back() { return p_[n_ - 1]; }
  const T& back() const { return p_[n_ - 1]; }
  void reserve(size_t c) { if (c > cap()) regrow(c); }
  template <class... A>
  T& emplace_back(A&&... a) {
    if (n_ == cap()) regrow(cap() ? 2 * cap() : 4);
    new (p_ + n_) T(std::forward<A>(a)...);
    return p_[n_++];
  }
  void push_back(const T& v) { emplace_back(v); }
  void push_back(T&& v) { emplace_back(std::move(v)); }
  void pop_back() { p_[--n_].~T(); }
  void clear() {
    for (uint32_t i = 0; i < n_; ++i) p_[i].~T();
    n_ = 0;
  }

 private:
  static constexpr uint32_t kArenaBit = 0x80000000u;
  T* p_ = nullptr;
  uint32_t n_ = 0;
  uint32_t cap_ = 0;                      // capacity | kArenaBit when the storage is arena memory
  size_t cap() const { return cap_ & ~kArenaBit; }
  bool in_arena() const { return (cap_ & kArenaBit) != 0; }
  // new storage: the arena when one is in scope and this vector is empty or
  // already arena-backed (a heap vector stays on the heap)
  T* allocate(size_t c, bool* arena) {
    Arena* a = current_arena();
    *arena = a && (p_ == nullptr || in_arena());
    return static_cast<T*>(*arena ? a->alloc(sizeof(T) * c) : ::operator new(sizeof(T) * c));
  }
  void regrow(size_t c) {
    if (c >= kArenaBit) throw std::bad_alloc();
    bool arena = false;
    T* q = allocate(c, &arena);
    for (uint32_t i = 0; i < n_; ++i) {
      new (q + i) T(std::move(p_[i]));
      p_[i].~T();
    }
    if (p_ && !in_arena()) ::operator delete(p_);
    p_ = q;
    cap_ = (uint32_t)c | (arena ? kArenaBit : 0u);
  }
  void destroy() {
    for (uint32_t i = 0; i < n_; ++i) p_[i].~T();
    if (p_ && !in_arena()) ::operator delete(p_);
    p_ = nullptr;
    n_ = cap_ = 0;
  }
  void copy_from(const Vec& o) {
    if (!o.n_) return;
    bool arena = false;
    p_ = allocate(o.n_, &arena);
    for (uint32_t i = 0; i < o.n_; ++i) new (p_ + i) T(o.p_[i]);
    n_ = o.n_;
    cap_ = o.n_ | (arena ? kArenaBit : 0u);
  }
  void take(Vec& o) {
    if (o.in_arena() && !current_arena()) {       // leaving the batch: to the heap
      if (o.n_) {
        p_ = static_cast<T*>(::operator new(sizeof(T) * o.n_));
        for (uint32_t i = 0; i < o.n_; ++i) new (p_ + i) T(std::move(o.p_[i]));
        n_ = cap_ = o.n_;
      }
      o.clear();
      o.p_ = nullptr;
      o.cap_ = 0;
      return;
    }
    p_ = o.p_; n_ = o.n_; cap_ = o.cap_;
    o.p_ = nullptr; o.n_ = o.cap_ = 0;
  }
};

// The text of a String / Number Value: up to 15 bytes inline, longer text on
// the heap -- or, for text the parser reads into a tree built under an arena
// scope (json::parse), in that arena.  Always NUL-terminated.  Moves follow
// Vec's rule: arena text leaving its batch (a move with no arena in scope) is
// copied to the heap.  A 1M-token batch's claim strings (issuer URLs,
// subjects) were ~1-3 mallocs and frees per token as std::string.
class Str {
 public:
  Str() { s_[0] = 0; }
  ~Str() { release(); }
  Str(const Str& o) : Str() { assign(o.data(), o.size()); }
  Str(Str&& o) noexcept : Str() { take(o); }
  explicit Str(std::string_view v) : Str() { assign(v.data(), v.size()); }
  Str& operator=(const Str& o) {
    if (this != &o) assign(o.data(), o.size());
    return *this;
  }
  Str& operator=(Str&& o) noexcept {
    if (this != &o) { release(); take(o); }
    return *this;
  }
  Str& operator=(std::string_view v) { assign(v.data(), v.size()); return *this; }
  void assign(const char* p, size_t n) { assign_in(nullptr, p, n); }
  void assign_in(Arena* a, const char* p, size_t n);   // a == nullptr: heap
  const char* data() const { return n_ <= kInline ? s_ : p_; }
  const char* c_str() const { return data(); }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  std::string_view view() const { return {data(), n_}; }
  operator std::string_view() const { return view(); }
  friend bool operator==(const Str& a, std::string_view b) { return a.view() == b; }
  friend bool operator!=(const Str& a, std::string_view b) { return a.view() != b; }

 private:
  static constexpr uint32_t kInline = 15;
  union {
    char s_[kInline + 1];
    char* p_;
  };
  uint32_t n_ = 0;
  bool arena_ = false;
  void release() {
    if (n_ > kInline && !arena_) ::operator delete(p_);
    n_ = 0;
    arena_ = false;
    s_[0] = 0;
  }
  void take(Str& o);
};

struct Value;
using Member = std::pair<std::string, Value>;

struct Value {
  enum Kind : uint8_t { Null, Bool, Number, String, Array, Object };
  Kind kind = Null;
  bool b = false;
  bool num_range_err = false;    // the literal overflows float64
  double num = 0;                // Number: float64 value (Go interface{} decoding)
  Str str;                       // String: decoded text; Number: the literal as written
  Vec<Value> arr;
  Vec<Member> obj;               // insertion order of first occurrence, last value wins

  const Value* get(std::string_view key) const;   // exact (case-sensitive) member lookup
  bool is_null() const { return kind == Null; }
};

// Parse a complete JSON text.  Returns false and sets *err on a syntax error
// (Go: "invalid character ..." / "unexpected end of JSON input").
bool parse(std::string_view text, Value* out, std::string* err);

// True iff the value (recursively) holds a number literal that does not fit a
// float64: unmarshalling it into interface{} fails in Go.
bool has_range_error(const Value& v);

// Serialise like Go's json.Marshal of the interface{} tree: object keys sorted
// bytewise, float64 formatted as encoding/json does ('f' unless the exponent
// is < -6 or >= 21), HTML-safe escapes (<, >, & as < ...).
std::string marshal(const Value& v);

// Go's strconv.FormatFloat(f, 'g'-style rule used by encoding/json floatEncoder.
std::string format_float(double f);

// utf8.DecodeRune: the rune at s[0..n) and its width; (0xFFFD, 1) when invalid.
uint32_t decode_rune(const unsigned char* s, size_t n, size_t* w);
void put_utf8(std::string& o, uint32_t r);

}  // namespace json
}  // namespace capjwt
