// degraded.cpp -- the key sets' degraded path with the device call failing
// (fault_stub.cpp): every token that needed the device gets the device error
// as its own error, the call itself returns; parse errors and "no key" misses
// keep their usual errors, and a JWKS key set does not refetch for a token
// whose device call failed.  Prints FAIL lines and exits 1 on a mismatch.
#include <cstdio>
#include <string>
#include <vector>

#include "../../cap_amd/csrc/host/cap_jwt.hpp"

using namespace capjwt;

static int fails = 0;
static void check(bool ok, const char* what, const std::string& got) {
  if (!ok) {
    std::printf("FAIL %s: %s\n", what, got.c_str());
    ++fails;
  }
}
static bool has(const std::string& s, const char* sub) { return s.find(sub) != std::string::npos; }

int main() {
  // {"alg":"EdDSA","kid":"k1"} . {"sub":"a"} . 64 zero bytes
  const std::string ed_tok =
      "eyJhbGciOiJFZERTQSIsImtpZCI6ImsxIn0.eyJzdWIiOiJhIn0." + std::string(86, 'A');
  // {"alg":"ES256"} . {"sub":"a"} . 64 zero bytes: no EC key in the set
  const std::string es_tok = "eyJhbGciOiJFUzI1NiJ9.eyJzdWIiOiJhIn0." + std::string(86, 'A');
  const std::vector<std::string_view> toks = {ed_tok, "not-a-jwt", es_tok};
  const char* dev = "capjwt: signature verification unavailable: capjwt: jg_verify_batch: hipErrorIllegalAddress";

  PublicKey ed;
  ed.kind = PublicKey::Ed25519;
  ed.x = std::string(32, '\0');
  std::string err;
  auto ks = NewStaticKeySet({ed}, &err);
  check(ks != nullptr, "static key set", err);
  Results r = ks->VerifySignatureBatch(toks);
  check(!r[0].ok && has(r[0].err, dev), "static: device error", r[0].err);
  check(!r[1].ok && !r[1].err.empty() && !has(r[1].err, "unavailable"), "static: parse error", r[1].err);
  check(!r[2].ok && r[2].err == "no known key successfully validated the token signature", "static: no key", r[2].err);

  auto v = NewValidator(ks.get(), &err);
  Expected ex;
  ex.SigningAlgorithms = {"EdDSA"};
  Results vr = v->ValidateBatch({ed_tok}, ex);
  check(!vr[0].ok && has(vr[0].err, dev), "validator: device error", vr[0].err);

  int fetches = 0;
  Fetcher f = [&](const std::string&, const std::string&) {
    ++fetches;
    FetchResponse resp;
    resp.body = R"({"keys":[{"kty":"OKP","crv":"Ed25519","kid":"k1","x":")" + std::string(43, 'A') + R"("}]})";
    return resp;                                           // max_age -1: expires at once
  };
  auto jw = NewJSONWebKeySet("https://issuer.example/keys", "", f, &err);
  check(jw != nullptr, "jwks key set", err);
  Results jr = jw->VerifySignatureBatch(toks);
  check(!jr[0].ok && has(jr[0].err, dev), "jwks: device error", jr[0].err);
  check(!jr[1].ok && has(jr[1].err, "oidc: malformed jwt: "), "jwks: parse error", jr[1].err);
  check(!jr[2].ok && jr[2].err == "failed to verify id token signature", "jwks: no key", jr[2].err);
  check(fetches == 1, "jwks: first call fetches once (empty cache)", std::to_string(fetches));
  // the cache has expired (max_age none), but a token whose device call failed
  // is no miss: no refetch
  jr = jw->VerifySignatureBatch({ed_tok});
  check(!jr[0].ok && has(jr[0].err, dev), "jwks: device error again", jr[0].err);
  check(fetches == 1, "jwks: no refetch for a device failure", std::to_string(fetches));
  // each failed call recreated the context (Engine::recover: new jg_ctx, the
  // key list re-staged from the key set's own copy, no refetch)
  check(jw->DeviceRecoveries() >= 2, "jwks: context recreated after each failure",
        std::to_string(jw->DeviceRecoveries()));
  check(jw->DeviceStatus().empty(), "jwks: healthy after recovery", jw->DeviceStatus());
  // a single-token call takes the coalescer and gets the same error
  Result one = jw->VerifySignature(ed_tok);
  check(!one.ok && has(one.err, dev), "jwks: coalesced single call", one.err);
  Result vone = v->Validate(ed_tok, ex);
  check(!vone.ok && has(vone.err, dev) && has(vone.err, "error verifying token signature: "), "validator: single",
        vone.err);
  // go-oidc adapter (remoteKeySet.VerifySignature, payload bytes)
  {
    auto rk = NewRemoteKeySet("https://issuer.example/keys", f);
    auto pr = rk->VerifySignatureBatch({ed_tok, "not-a-jwt"});
    check(!pr[0].ok && has(pr[0].err, dev), "remote: device error", pr[0].err);
    check(!pr[1].ok && has(pr[1].err, "oidc: malformed jwt: "), "remote: parse error", pr[1].err);
  }
  // oidc hash claims: a failed jg_hash_batch becomes each pair's error
  {
    Engine eng({});
    // {"alg":"RS256"} . {"at_hash":"x"} . "AAAA"
    const std::string idt = "eyJhbGciOiJSUzI1NiJ9.eyJhdF9oYXNoIjoieCJ9.AAAA";
    auto hr = VerifyAccessTokenBatch(eng, {idt, "not-a-jwt"}, {"access-token", "access-token"});
    check(!hr[0].verified && has(hr[0].err, "VerifyAccessToken: capjwt: hash unavailable: capjwt: jg_hash_batch: "),
          "hash: device error", hr[0].err);
    check(!hr[1].verified && !hr[1].err.empty() && !has(hr[1].err, "unavailable"), "hash: parse error", hr[1].err);
  }
  std::printf(fails ? "degraded: %d failures\n" : "degraded: ok\n", fails);
  return fails ? 1 : 0;
}
