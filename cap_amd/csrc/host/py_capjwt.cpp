// py_capjwt.cpp -- Python binding of the C++ cap jwt mirror (cap_jwt.hpp), so
// the parity tests can drive KeySet / Validator the way the reference's Go
// tests do (jwt/keyset_test.go, jwt/jwt_test.go).  Values cross as Go would
// hand them out: claims map -> dict with float64 numbers; error -> str or None.
#include <pybind11/functional.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "cap_jwt.hpp"

namespace py = pybind11;
using namespace capjwt;

namespace {

py::object to_py(const json::Value& v) {
  switch (v.kind) {
    case json::Value::Null: return py::none();
    case json::Value::Bool: return py::bool_(v.b);
    case json::Value::Number: return py::float_(v.num);
    case json::Value::String: return py::str(v.str.data(), v.str.size());
    case json::Value::Array: {
      py::list l;
      for (const auto& e : v.arr) l.append(to_py(e));
      return std::move(l);
    }
    case json::Value::Object: {
      py::dict d;
      for (const auto& m : v.obj) d[py::str(m.first)] = to_py(m.second);
      return std::move(d);
    }
  }
  return py::none();
}

py::tuple result_py(const Result& r) {
  if (r.ok) return py::make_tuple(to_py(r.claims), py::none());
  return py::make_tuple(py::none(), py::str(r.err));
}

py::list results_py(const Results& rs) {
  py::list l;
  for (const auto& r : rs) l.append(result_py(r));
  return l;
}

std::vector<std::string> as_strings(const py::sequence& toks) {
  std::vector<std::string> v;
  v.reserve(py::len(toks));
  for (auto t : toks) {
    if (py::isinstance<py::bytes>(t)) v.push_back(t.cast<std::string>());
    else v.push_back(t.cast<std::string>());
  }
  return v;
}

std::vector<std::string_view> views(const std::vector<std::string>& s) {
  return std::vector<std::string_view>(s.begin(), s.end());
}

// newline-separated token blob -> views (end-to-end benchmark input, no
// per-token Python objects).  One thread: a parallel split measured 4-5x
// slower on the GPU box (16-CPU cgroup quota: a 16-thread burst next to the
// runtime's own threads is throttled for the rest of the CFS period).
void split_range(const char* p, const char* end, std::vector<std::string_view>& v) {
  while (p < end) {
    const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
    const char* e = nl ? nl : end;
    if (e > p) v.emplace_back(p, (size_t)(e - p));
    p = e + 1;
  }
}

// newline-separated tokens -> views; a large blob is cut at newlines into one
// range per host thread (a 1M-token blob: 9 ms on one thread)
std::vector<std::string_view> split_lines(const char* p, size_t n) {
  const size_t th = n >= (size_t(64) << 20) ? (size_t)capjwt::host_threads() : 1;
  std::vector<const char*> cut{p};
  for (size_t t = 1; t < th; ++t) {
    const char* c = p + n * t / th;
    const char* nl = static_cast<const char*>(std::memchr(c, '\n', (size_t)(p + n - c)));
    cut.push_back(nl && nl + 1 > cut.back() ? nl + 1 : cut.back());
  }
  cut.push_back(p + n);
  std::vector<std::vector<std::string_view>> part(cut.size() - 1);
  auto run = [&](size_t k) {
    part[k].reserve((size_t)(cut[k + 1] - cut[k]) / 256 + 1);
    split_range(cut[k], cut[k + 1], part[k]);
  };
  std::vector<std::thread> ths;
  for (size_t k = 1; k < part.size(); ++k) ths.emplace_back(run, k);
  run(0);
  for (auto& t : ths) t.join();
  if (part.size() == 1) return std::move(part[0]);
  size_t total = 0;
  for (auto& x : part) total += x.size();
  std::vector<std::string_view> v;
  v.reserve(total);
  for (auto& x : part) v.insert(v.end(), x.begin(), x.end());
  return v;
}

Fetcher wrap_fetch(py::object fn) {
  // fn(url, ca_pem) -> dict(status=, status_text=, body=, content_type=, max_age=); raise = transport error
  auto holder = std::make_shared<py::object>(std::move(fn));
  return [holder](const std::string& url, const std::string& ca) -> FetchResponse {
    py::gil_scoped_acquire g;
    FetchResponse r;
    py::object res;
    try {
      res = (*holder)(url, ca);
    } catch (py::error_already_set& e) {
      throw std::runtime_error(std::string("Get \"") + url + "\": " + e.what());
    }
    py::dict d = res.cast<py::dict>();
    if (d.contains("status")) r.status = d["status"].cast<int>();
    r.status_text = d.contains("status_text") ? d["status_text"].cast<std::string>()
                                              : std::to_string(r.status) + (r.status == 200 ? " OK" : "");
    if (d.contains("body")) {
      py::object b = d["body"];
      r.body = py::isinstance<py::bytes>(b) ? b.cast<std::string>() : b.cast<std::string>();
    }
    if (d.contains("content_type")) r.content_type = d["content_type"].cast<std::string>();
    if (d.contains("max_age")) r.max_age_s = d["max_age"].cast<int64_t>();
    return r;
  };
}

struct PyKeySet {
  std::shared_ptr<KeySet> ks;
};

PyKeySet must(std::unique_ptr<KeySet> p, const std::string& err) {
  if (!p) throw py::value_error(err);
  return PyKeySet{std::shared_ptr<KeySet>(std::move(p))};
}

py::dict key_dict(const PublicKey& k) {
  py::dict d;
  static const char* kinds[] = {"none", "RSA", "EC", "Ed25519", "oct"};
  d["kind"] = kinds[k.kind];
  if (k.kind == PublicKey::RSA) {
    d["n"] = py::bytes(k.n);
    d["e"] = k.e;
  } else if (k.kind == PublicKey::EC) {
    static const char* crv[] = {"", "P-256", "P-384", "P-521"};
    d["crv"] = crv[k.curve];
    d["x"] = py::bytes(k.x);
    d["y"] = py::bytes(k.y);
  } else if (k.kind == PublicKey::Ed25519) {
    d["x"] = py::bytes(k.x);
  } else if (k.kind == PublicKey::Symmetric) {
    d["k"] = py::bytes(k.k);
  }
  return d;
}

}  // namespace

PYBIND11_MODULE(_capjwt_host, m) {
  m.doc() = "C++ host mirror of cap's jwt package over the MI355X verifier (libcapjwt.so)";

  py::class_<PublicKey>(m, "PublicKey")
      .def_static("rsa", [](py::bytes n, uint64_t e) {
        PublicKey k;
        k.kind = PublicKey::RSA;
        std::string s = n;
        size_t i = 0;
        while (i < s.size() && s[i] == 0) ++i;
        k.n = s.substr(i);
        k.e = e;
        return k;
      })
      .def_static("ec", [](const std::string& crv, py::bytes x, py::bytes y) {
        PublicKey k;
        k.kind = PublicKey::EC;
        k.curve = crv == "P-256" ? 1 : crv == "P-384" ? 2 : crv == "P-521" ? 3 : 0;
        if (!k.curve) throw py::value_error("unsupported curve " + crv);
        k.x = x;
        k.y = y;
        return k;
      })
      .def_static("ed25519", [](py::bytes pub) {
        PublicKey k;
        k.kind = PublicKey::Ed25519;
        k.x = pub;
        return k;
      })
      .def_static("symmetric", [](py::bytes secret) {
        PublicKey k;
        k.kind = PublicKey::Symmetric;
        k.k = secret;
        return k;
      })
      .def("as_dict", &key_dict)
      .def("__eq__", [](const PublicKey& a, const PublicKey& b) { return a == b; });

  py::class_<Expected>(m, "Expected")
      .def(py::init<>())
      .def_readwrite("Issuer", &Expected::Issuer)
      .def_readwrite("Subject", &Expected::Subject)
      .def_readwrite("ID", &Expected::ID)
      .def_readwrite("Audiences", &Expected::Audiences)
      .def_readwrite("SigningAlgorithms", &Expected::SigningAlgorithms)
      .def_readwrite("NotBeforeLeeway", &Expected::NotBeforeLeeway)
      .def_readwrite("ExpirationLeeway", &Expected::ExpirationLeeway)
      .def_readwrite("ClockSkewLeeway", &Expected::ClockSkewLeeway)
      .def_readwrite("has_now", &Expected::has_now)
      .def_readwrite("now_unix_ns", &Expected::now_unix_ns);

  // ---- CPU-side pieces (no GPU needed)
  m.def("supported_signing_algorithm", [](const std::vector<std::string>& algs) -> py::object {
    const std::string e = SupportedSigningAlgorithm(algs);
    if (e.empty()) return py::none();
    return py::str(e);
  });
  m.def("json_loads", [](py::bytes b) -> py::tuple {
    json::Value v;
    std::string err;
    std::string s = b;
    if (!json::parse(s, &v, &err)) return py::make_tuple(py::none(), py::str(err));
    if (json::has_range_error(v)) return py::make_tuple(py::none(), py::str("number out of range"));
    return py::make_tuple(to_py(v), py::none());
  });
  m.def("json_marshal", [](py::bytes b) -> py::object {
    // json.Marshal of the parsed interface{} (sorted keys; a member appears once)
    json::Value v;
    std::string err, s = b;
    if (!json::parse(s, &v, &err)) return py::none();
    return py::bytes(json::marshal(v));
  });
  m.def("b64url_decode", [](const std::string& s) -> py::object {
    std::string out, err;
    if (!b64url_decode(s, &out, &err)) return py::none();
    return py::bytes(out);
  });
  m.def("strip_whitespace", [](py::bytes s) { return py::bytes(strip_whitespace(std::string(s))); });
  m.def("parse_signed", [](py::bytes tok) -> py::dict {
    JWS j;
    std::string err;
    py::dict d;
    std::string t = tok;
    if (!parse_signed(t, &j, &err)) {
      d["error"] = err;
      return d;
    }
    d["error"] = py::none();
    d["payload"] = py::bytes(j.payload);
    d["nsigs"] = j.sigs.size();
    if (!j.sigs.empty()) {
      d["alg"] = j.sigs[0].alg;
      d["kid"] = j.sigs[0].kid;
      d["signature"] = py::bytes(j.sigs[0].signature);
      d["protected"] = py::bytes(j.sigs[0].protected_raw);
    }
    std::string si;
    if (signing_input(j, &si)) d["signing_input"] = py::bytes(si);
    else d["signing_input"] = py::none();
    return d;
  });
  m.def("parse_public_key_pem", [](py::bytes pem) {
    PublicKey k;
    std::string err;
    if (!ParsePublicKeyPEM(std::string(pem), &k, &err)) throw py::value_error(err);
    return k;
  });
  m.def("jwks_decode", [](py::bytes doc) {
    std::vector<JSONWebKey> keys;
    std::string err;
    if (!jwks_decode(std::string(doc), &keys, &err)) throw py::value_error(err);
    py::list l;
    for (const auto& k : keys) l.append(py::make_tuple(k.kid, k.key));
    return l;
  });
  m.def("ec_on_curve", [](const std::string& crv, py::bytes x, py::bytes y) {
    const int c = crv == "P-256" ? 1 : crv == "P-384" ? 2 : crv == "P-521" ? 3 : 0;
    return ec_on_curve(c, std::string(x), std::string(y));
  });
  m.def("validate_claims", [](py::bytes payload, const std::string& alg, size_t sig_len, const Expected& exp,
                              int64_t now_ns) {
    // the post-signature half of Validate on a payload whose signature verified
    json::Value v;
    std::string err;
    if (!json::parse(std::string(payload), &v, &err)) return py::tuple(py::make_tuple(py::none(), py::str(err)));
    TokenInfo info;
    info.parsed = true;
    info.nsigs = 1;
    info.sig0_len = sig_len;
    info.alg = alg;
    Result r = validate_claims(v, info, exp, now_ns);
    if (r.ok) r.claims = v;
    return result_py(r);
  });
  m.def("host_threads", &host_threads);
  m.def("set_host_memory_retention", &SetHostMemoryRetention);
  m.def("trim_host_memory", &TrimHostMemory);
  m.def("host_memory_retained", &HostMemoryRetained);
  m.def("available_cpus", &available_cpus);

  // ---- GPU-backed key sets and validator
  py::class_<PyKeySet>(m, "KeySet")
      .def("verify_signature", [](PyKeySet& s, py::object tok) {
        std::string t = tok.cast<std::string>();
        Result r;
        {
          py::gil_scoped_release rel;
          r = s.ks->VerifySignature(t);
        }
        return result_py(r);
      })
      .def("verify_signature_batch", [](PyKeySet& s, py::sequence toks) {
        auto v = as_strings(toks);
        Results rs;
        {
          py::gil_scoped_release rel;
          rs = s.ks->VerifySignatureBatch(views(v));
        }
        return results_py(rs);
      })
      .def("wait_tables", [](PyKeySet& s) {
        py::gil_scoped_release rel;
        s.ks->WaitTables();
      })
      .def("set_coalescing", [](PyKeySet& s, int max_inflight, size_t max_batch, int64_t window_us) {
        CoalesceConfig c;
        c.max_inflight = max_inflight;
        c.max_batch = max_batch;
        c.window_us = window_us;
        s.ks->SetCoalescing(c);
      }, py::arg("max_inflight") = 2, py::arg("max_batch") = 65536, py::arg("window_us") = 0)
      .def("coalescing_stats", [](PyKeySet& s) {
        const auto st = s.ks->CoalescingStats();
        py::dict d;
        d["calls"] = st.calls;
        d["batches"] = st.batches;
        d["max_batch"] = st.max_batch_seen;
        return d;
      })
      .def("device_status", [](PyKeySet& s) {
        py::gil_scoped_release rel;
        return s.ks->DeviceStatus();
      })
      .def("device_recoveries", [](PyKeySet& s) { return s.ks->DeviceRecoveries(); })
      .def("_debug_fail_verify", [](PyKeySet& s, int n) {
        if (s.ks->DebugFailVerify(n) != 0) throw py::value_error("jg_debug_fail_verify failed");
      });

  m.def("new_static_keyset", [](const std::vector<PublicKey>& keys, const std::vector<int>& devices) {
    std::string err;
    return must(NewStaticKeySet(keys, &err, devices), err);
  }, py::arg("keys"), py::arg("devices") = std::vector<int>{});
  m.def("new_json_web_keyset", [](const std::string& url, const std::string& ca, py::object fetch,
                                  const std::vector<int>& devices) {
    std::string err;
    return must(NewJSONWebKeySet(url, ca, wrap_fetch(std::move(fetch)), &err, devices), err);
  }, py::arg("url"), py::arg("ca_pem"), py::arg("fetch"), py::arg("devices") = std::vector<int>{});
  m.def("new_oidc_discovery_keyset", [](const std::string& issuer, const std::string& ca, py::object fetch,
                                        const std::vector<int>& devices) {
    std::string err;
    std::unique_ptr<KeySet> ks;
    {
      ks = NewOIDCDiscoveryKeySet(issuer, ca, wrap_fetch(std::move(fetch)), &err, devices);
    }
    return must(std::move(ks), err);
  }, py::arg("issuer"), py::arg("ca_pem"), py::arg("fetch"), py::arg("devices") = std::vector<int>{});

  struct PyValidator {
    std::shared_ptr<KeySet> ks;
    std::unique_ptr<Validator> v;
  };
  py::class_<PyValidator>(m, "Validator")
      .def(py::init([](PyKeySet* ks) {
        if (!ks) throw py::value_error("keySet must not be nil");
        auto p = std::make_unique<PyValidator>();
        p->ks = ks->ks;
        p->v = std::make_unique<Validator>(ks->ks.get());
        return p;
      }))
      .def("validate", [](PyValidator& s, py::object tok, const Expected& e) {
        std::string t = tok.cast<std::string>();
        Result r;
        {
          py::gil_scoped_release rel;
          r = s.v->Validate(t, e);
        }
        return result_py(r);
      })
      .def("validate_batch", [](PyValidator& s, py::sequence toks, const Expected& e) {
        auto v = as_strings(toks);
        Results rs;
        {
          py::gil_scoped_release rel;
          rs = s.v->ValidateBatch(views(v), e);
        }
        return results_py(rs);
      })
      .def("validate_blob", [](PyValidator& s, py::bytes blob, const Expected& e) {
        // end-to-end throughput entry: newline-separated tokens in, per-token
        // accept bytes out (claims stay on the C++ side)
        // zero-copy: the bytes object is immutable and stays referenced by the
        // caller for the duration of the call
        char* bp = nullptr;
        Py_ssize_t bn = 0;
        if (PyBytes_AsStringAndSize(blob.ptr(), &bp, &bn) != 0) throw py::error_already_set();
        std::string ok;
        {
          py::gil_scoped_release rel;
          const bool trace = std::getenv("CAPJWT_TRACE") != nullptr;
          auto t0 = std::chrono::steady_clock::now();
          auto lap = [&](const char* what) {
            if (!trace) return;
            const auto t1 = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[capjwt] blob %-12s %8.2f ms\n", what,
                         std::chrono::duration<double, std::milli>(t1 - t0).count());
            t0 = t1;
          };
          auto toks = split_lines(bp, (size_t)bn);
          lap("split");
          auto rs = s.v->ValidateBatch(toks, e);
          lap("validate");
          ok.resize(rs.size());
          for (size_t i = 0; i < rs.size(); ++i) ok[i] = rs[i].ok ? 1 : 0;
          release_results(rs);
          lap("release");
        }
        return py::bytes(ok);
      })
      .def("_concurrent_validate", [](PyValidator& s, py::bytes blob, const Expected& e, int callers,
                                      int64_t total, int pin_cpus) {
        // Measurement helper (bench.py `single`): `callers` host threads, each
        // calling Validator::Validate once per token -- the goroutine-per-
        // request pattern of an unchanged cap caller -- over `total` tokens
        // taken round-robin from the newline-separated pool.  Returns the
        // wall time, accepts and per-call latency percentiles.
        char* bp = nullptr;
        Py_ssize_t bn = 0;
        if (PyBytes_AsStringAndSize(blob.ptr(), &bp, &bn) != 0) throw py::error_already_set();
        callers = std::max(1, callers);
        std::vector<std::vector<int64_t>> lat(callers);
        std::vector<int64_t> acc(callers, 0);
        double wall = 0;
        {
          py::gil_scoped_release rel;
          const auto toks = split_lines(bp, (size_t)bn);
          if (toks.empty()) throw std::runtime_error("empty token pool");
          std::atomic<int64_t> next{0};
          std::vector<std::thread> th;
          // pin_cpus > 0: every caller thread runs on the first pin_cpus CPUs the
          // process may use (a Go service's goroutines on GOMAXPROCS threads)
          cpu_set_t pin;
          CPU_ZERO(&pin);
          if (pin_cpus > 0) {
            cpu_set_t all;
            CPU_ZERO(&all);
            if (sched_getaffinity(0, sizeof all, &all) == 0) {
              int k = 0;
              for (int c = 0; c < CPU_SETSIZE && k < pin_cpus; ++c)
                if (CPU_ISSET(c, &all)) { CPU_SET(c, &pin); ++k; }
            }
          }
          const auto t0 = std::chrono::steady_clock::now();
          for (int c = 0; c < callers; ++c)
            th.emplace_back([&, c] {
              if (pin_cpus > 0 && CPU_COUNT(&pin) > 0) (void)sched_setaffinity(0, sizeof pin, &pin);
              lat[c].reserve((size_t)(total / callers + 16));
              while (true) {
                const int64_t i = next.fetch_add(1);
                if (i >= total) break;
                const auto a = std::chrono::steady_clock::now();
                Result r = s.v->Validate(toks[(size_t)i % toks.size()], e);
                const auto b = std::chrono::steady_clock::now();
                lat[c].push_back(std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count());
                acc[c] += r.ok;
              }
            });
          for (auto& t : th) t.join();
          wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        std::vector<int64_t> all;
        for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
        std::sort(all.begin(), all.end());
        auto pct = [&](double q) { return all.empty() ? 0.0 : (double)all[std::min(all.size() - 1, (size_t)(q * (double)all.size()))] / 1e3; };
        int64_t accepted = 0;
        for (auto a : acc) accepted += a;
        py::dict d;
        d["wall_s"] = wall;
        d["calls"] = (int64_t)all.size();
        d["accepted"] = accepted;
        d["p50_us"] = pct(0.50);
        d["p90_us"] = pct(0.90);
        d["p99_us"] = pct(0.99);
        d["p999_us"] = pct(0.999);
        d["max_us"] = all.empty() ? 0.0 : (double)all.back() / 1e3;
        return d;
      }, py::arg("blob"), py::arg("expected"), py::arg("callers"), py::arg("total"), py::arg("pin_cpus") = 0);

  // ---- go-oidc oidc.KeySet adapter (NewRemoteKeySet): payload bytes out
  struct PyRemoteKeySet {
    std::unique_ptr<RemoteKeySet> ks;
  };
  auto payload_py = [](const PayloadResult& r) {
    return py::make_tuple(r.ok ? py::object(py::bytes(r.payload)) : py::object(py::none()),
                          r.ok ? py::object(py::none()) : py::object(py::str(r.err)));
  };
  py::class_<PyRemoteKeySet>(m, "RemoteKeySet")
      .def("verify_signature", [payload_py](PyRemoteKeySet& s, py::object tok) {
        std::string t = tok.cast<std::string>();
        PayloadResult r;
        {
          py::gil_scoped_release rel;
          r = s.ks->VerifySignature(t);
        }
        return payload_py(r);
      })
      .def("verify_signature_batch", [payload_py](PyRemoteKeySet& s, py::sequence toks) {
        auto v = as_strings(toks);
        std::vector<PayloadResult> rs;
        {
          py::gil_scoped_release rel;
          rs = s.ks->VerifySignatureBatch(views(v));
        }
        py::list out;
        for (const auto& r : rs) out.append(payload_py(r));
        return out;
      })
      .def("set_coalescing", [](PyRemoteKeySet& s, int max_inflight, size_t max_batch, int64_t window_us) {
        CoalesceConfig c;
        c.max_inflight = max_inflight;
        c.max_batch = max_batch;
        c.window_us = window_us;
        s.ks->SetCoalescing(c);
      }, py::arg("max_inflight") = 2, py::arg("max_batch") = 65536, py::arg("window_us") = 0);
  m.def("new_remote_keyset", [](const std::string& url, py::object fetch, const std::vector<int>& devices) {
    auto p = std::make_unique<PyRemoteKeySet>();
    p->ks = NewRemoteKeySet(url, wrap_fetch(std::move(fetch)), devices);
    return p;
  }, py::arg("url"), py::arg("fetch"), py::arg("devices") = std::vector<int>{});

  // ---- oidc at_hash / c_hash (oidc/id_token.go:59-145) over one GPU context
  struct PyHashEngine {
    std::unique_ptr<Engine> eng;
  };
  auto hash_claims = [](PyHashEngine& s, py::sequence ids, py::sequence vals, bool code) {
    auto a = as_strings(ids), b = as_strings(vals);
    if (a.size() != b.size()) throw py::value_error("id_tokens and values differ in length");
    std::vector<HashClaimResult> rs;
    {
      py::gil_scoped_release rel;
      rs = code ? VerifyAuthorizationCodeBatch(*s.eng, views(a), views(b))
                : VerifyAccessTokenBatch(*s.eng, views(a), views(b));
    }
    py::list out;
    for (const auto& r : rs)
      out.append(py::make_tuple(r.verified, r.err.empty() ? py::object(py::none()) : py::object(py::str(r.err))));
    return out;
  };
  py::class_<PyHashEngine>(m, "HashEngine")
      .def(py::init([](const std::vector<int>& devices) {
        auto p = std::make_unique<PyHashEngine>();
        p->eng = std::make_unique<Engine>(devices);
        return p;
      }), py::arg("devices") = std::vector<int>{})
      .def("verify_access_token_batch", [hash_claims](PyHashEngine& s, py::sequence ids, py::sequence ats) {
        return hash_claims(s, ids, ats, false);
      })
      .def("verify_authorization_code_batch", [hash_claims](PyHashEngine& s, py::sequence ids, py::sequence codes) {
        return hash_claims(s, ids, codes, true);
      });
}
