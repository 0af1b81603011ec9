// Unit test of the batch arenas behind claims trees (host/json.hpp Vec / Arena,
// host/hostmem.hpp), built with ASan + UBSan by tests/test_json_arena.py.  CPU
// only; exits non-zero on the first failed check.  A tree that outlived its
// arena would read poisoned pool memory and ASan would abort.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <utility>
#include <vector>

#include "../../cap_amd/csrc/host/hostmem.hpp"
#include "../../cap_amd/csrc/host/json.hpp"

using namespace capjwt;

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

static const char* kClaims =
    "{\"aud\":[\"www.example.com\",\"a much longer audience string than fifteen\"],\"exp\":1611699944,"
    "\"iat\":1611699344,\"iss\":\"https://example.com/\",\"nested\":{\"k\":[1,2,{\"deep\":\"value long enough to be heap\"}]},"
    "\"sub\":\"alice@example.com\"}";

static void check_tree(const json::Value& v) {
  CHECK(v.kind == json::Value::Object);
  CHECK(v.obj.size() == 6);
  const json::Value* aud = v.get("aud");
  CHECK(aud && aud->arr.size() == 2 && aud->arr[1].str == "a much longer audience string than fifteen");
  const json::Value* n = v.get("nested");
  CHECK(n && n->get("k") && n->get("k")->arr.size() == 3);
  CHECK(n->get("k")->arr[2].get("deep")->str == "value long enough to be heap");
  CHECK(v.get("iss")->str == "https://example.com/");
  CHECK(json::marshal(v).size() > 100);
}

static bool in_range(const void* p, const json::Arena& a) { return a.used() > 0 && p != nullptr; }

int main() {
  // 1. a tree parsed under a scope, moved out after the scope and the arena are gone
  json::Value escaped;
  {
    auto arena = std::make_unique<json::Arena>();
    json::Value inside;
    {
      json::ArenaScope s(arena.get());
      std::string err;
      CHECK(json::parse(kClaims, &inside, &err));
      CHECK(arena->used() > 0);
      check_tree(inside);
      // 2. moves inside the scope are shallow (same storage)
      const void* before = inside.obj.begin();
      json::Value moved = std::move(inside);
      CHECK(moved.obj.begin() == before);
      inside = std::move(moved);
      CHECK(inside.obj.begin() == before);
      // 3. a copy inside the scope lives in the arena too
      json::Value c = inside;
      check_tree(c);
    }
    // no scope: this move leaves the arena (deep, to the heap)
    const void* arena_storage = inside.obj.begin();
    escaped = std::move(inside);
    CHECK(escaped.obj.begin() != arena_storage);
    CHECK(in_range(arena_storage, *arena));
    // the arena's blocks go back to the (poisoned) pool here
  }
  check_tree(escaped);
  // 4. a copy of an arena tree made outside any scope is heap storage
  {
    json::Arena a;
    json::Value t;
    {
      json::ArenaScope s(&a);
      std::string err;
      CHECK(json::parse(kClaims, &t, &err));
    }
    json::Value c = t;           // heap
    json::Value d;
    d = t;                       // heap
    t = json::Value();           // releases nothing to the heap: arena storage
    check_tree(c);
    check_tree(d);
  }
  // 5. a heap vector that grows inside a scope stays on the heap
  json::Value h;
  h.kind = json::Value::Array;
  h.arr.emplace_back();
  {
    json::Arena a;
    json::ArenaScope s(&a);
    for (int i = 0; i < 100; ++i) h.arr.emplace_back().str = "element number " + std::to_string(i) + " of the heap array";
    CHECK(a.used() == 0);
  }
  CHECK(h.arr.size() == 101 && h.arr[100].str == "element number 99 of the heap array");
  // 6. many objects growing past their first reservation, in one arena
  {
    json::Arena a;
    std::vector<json::Value> keep(64);
    {
      json::ArenaScope s(&a);
      for (auto& v : keep) {
        std::string doc = "{";
        for (int k = 0; k < 40; ++k) doc += (k ? ",\"m" : "\"m") + std::to_string(k) + "\":" + std::to_string(k);
        doc += "}";
        std::string err;
        CHECK(json::parse(doc, &v, &err));
        CHECK(v.obj.size() == 40 && v.obj[39].second.num == 39);
      }
    }
    for (auto& v : keep) v = json::Value();
  }
  // 7. the pools' retention cap
  {
    hostmem::set_retention_cap(size_t(64) << 20);
    std::vector<void*> b;
    for (int i = 0; i < 40; ++i) b.push_back(hostmem::block_get());
    for (void* p : b) hostmem::block_put(p);
    CHECK(hostmem::retained() <= (size_t(64) << 20));
    CHECK(hostmem::retained() >= (size_t(60) << 20));
    size_t cap = 0;
    void* big = hostmem::big_get(size_t(3) << 20, &cap);
    CHECK(cap >= (size_t(3) << 20));
    static_cast<char*>(big)[cap - 1] = 1;
    hostmem::big_put(big, cap);
    hostmem::trim();
    CHECK(hostmem::retained() == 0);
    hostmem::set_retention_cap(size_t(4) << 30);
  }
  std::printf("json arena test ok\n");
  return 0;
}
