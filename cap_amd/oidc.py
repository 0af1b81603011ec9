"""cap's oidc id_token hash-claim checks, backed by the MI355X SHA-2 kernel.

    Go (reference)                                        here
    IDToken.VerifyAccessToken        oidc/id_token.go:59   IDToken.VerifyAccessToken (+ VerifyAccessTokenBatch)
    IDToken.VerifyAuthorizationCode  oidc/id_token.go:83   IDToken.VerifyAuthorizationCode (+ VerifyAuthorizationCodeBatch)

Host work (UnmarshalClaims, go-jose ParseSigned, the alg checks, base64url)
runs in the C++ host mirror (cap_amd/csrc/host/cap_jwt.hpp); the hashes of a
batch run in one jg_hash_batch on the GPU.  Go's `(bool, error)` becomes
`(verified, err)` with err a str or None; the strings are the reference's.
"""
import threading
from typing import List, Optional, Sequence, Tuple

from . import _lib  # noqa: F401  (loads libcapjwt.so first; fails loudly if missing)
from . import _capjwt_host as _h

_engine = None
_engine_lock = threading.Lock()


def _eng():
    global _engine
    with _engine_lock:
        if _engine is None:
            _engine = _h.HashEngine()
        return _engine


def _b(v) -> bytes:
    return v if isinstance(v, bytes) else str(v).encode()


def VerifyAccessTokenBatch(id_tokens: Sequence, access_tokens: Sequence) -> List[Tuple[bool, Optional[str]]]:
    """IDToken(id_tokens[i]).VerifyAccessToken(access_tokens[i]) for every i, one GPU batch."""
    return _eng().verify_access_token_batch([_b(t) for t in id_tokens], [_b(a) for a in access_tokens])


def VerifyAuthorizationCodeBatch(id_tokens: Sequence, codes: Sequence) -> List[Tuple[bool, Optional[str]]]:
    """IDToken(id_tokens[i]).VerifyAuthorizationCode(codes[i]) for every i, one GPU batch."""
    return _eng().verify_authorization_code_batch([_b(t) for t in id_tokens], [_b(c) for c in codes])


class IDToken(str):
    """oidc.IDToken (oidc/id_token.go:16)."""

    def VerifyAccessToken(self, access_token) -> Tuple[bool, Optional[str]]:
        return tuple(VerifyAccessTokenBatch([str(self)], [access_token])[0])

    def VerifyAuthorizationCode(self, code) -> Tuple[bool, Optional[str]]:
        return tuple(VerifyAuthorizationCodeBatch([str(self)], [code])[0])


AccessToken = str


class RemoteKeySet:
    """go-oidc v2.2.1 `oidc.KeySet` from oidc.NewRemoteKeySet: VerifySignature
    returns the verified payload bytes.  This is the interface cap's
    jsonWebKeySet wraps (jwt/keyset.go:101,120,127) and go-oidc's ID token
    verifier calls behind cap's Provider.VerifyIDToken (oidc/provider.go:418-441);
    here every signature check is the GPU verifier's."""

    def __init__(self, impl):
        self._impl = impl

    def VerifySignature(self, ctx, jwt) -> Tuple[Optional[bytes], Optional[str]]:
        return tuple(self._impl.verify_signature(jwt))

    def VerifySignatureBatch(self, ctx, jwts: Sequence) -> List[Tuple[Optional[bytes], Optional[str]]]:
        return [tuple(r) for r in self._impl.verify_signature_batch(list(jwts))]


def NewRemoteKeySet(ctx, jwks_url: str, fetch=None, devices=()) -> RemoteKeySet:
    """oidc.NewRemoteKeySet(ctx, jwksURL); `fetch(url, ca_pem)` stands in for
    the context's HTTP client (see cap_amd.jwt)."""
    return RemoteKeySet(_h.new_remote_keyset(jwks_url, fetch, list(devices)))
