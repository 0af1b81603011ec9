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
#include <memory>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace capjwt {
namespace json {

struct Value;
using Member = std::pair<std::string, Value>;

struct Value {
  enum Kind : uint8_t { Null, Bool, Number, String, Array, Object };
  Kind kind = Null;
  bool b = false;
  double num = 0;                // Number: float64 value (Go interface{} decoding)
  bool num_range_err = false;    // the literal overflows float64
  std::string str;               // String: decoded text; Number: the literal as written
  std::vector<Value> arr;
  std::vector<Member> obj;       // insertion order of first occurrence, last value wins

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
