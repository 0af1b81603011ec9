"""cap's jwt package API, backed by the MI355X verifier.

Mirrors the Go reference one to one (same names, argument meaning, error
strings); every call goes to the C++ host mirror (cap_amd/csrc/host/cap_jwt.hpp)
and every signature check to libcapjwt.so on the GPU.  Go's `(value, error)`
returns become `(value, err)` tuples with `err` a str or None.

    Go (reference)                                  here
    jwt.NewStaticKeySet      jwt/keyset.go:142       NewStaticKeySet
    jwt.NewJSONWebKeySet     jwt/keyset.go:109       NewJSONWebKeySet
    jwt.NewOIDCDiscoveryKeySet jwt/keyset.go:49      NewOIDCDiscoveryKeySet
    KeySet.VerifySignature   jwt/keyset.go:27-32     KeySet.VerifySignature (+ VerifySignatureBatch)
    jwt.ParsePublicKeyPEM    jwt/keyset.go:178       ParsePublicKeyPEM
    jwt.NewValidator         jwt/jwt.go:25           NewValidator
    Validator.Validate       jwt/jwt.go:95           Validator.Validate (+ ValidateBatch, north star)
    jwt.Expected             jwt/jwt.go:38           Expected
    jwt.SupportedSigningAlgorithm jwt/algs.go:38     SupportedSigningAlgorithm

HTTP is the caller's: NewJSONWebKeySet / NewOIDCDiscoveryKeySet take a
`fetch(url, ca_pem) -> {"status", "body", "content_type", "max_age"}` callable
standing in for the reference's net/http client (raise for a transport error).
"""
import dataclasses
import datetime
from typing import Callable, List, Optional, Sequence

from . import _lib  # noqa: F401  (loads libcapjwt.so first; fails loudly if missing)
from . import _capjwt_host as _h

# jwt/algs.go:12-21
RS256, RS384, RS512 = "RS256", "RS384", "RS512"
ES256, ES384, ES512 = "ES256", "ES384", "ES512"
PS256, PS384, PS512 = "PS256", "PS384", "PS512"
EdDSA = "EdDSA"
DefaultLeewaySeconds = 150          # jwt/jwt.go:16

PublicKey = _h.PublicKey


def SupportedSigningAlgorithm(*algs) -> Optional[str]:
    """jwt/algs.go:38-46: None, or `unsupported signing algorithm "X"`."""
    return _h.supported_signing_algorithm(list(algs))


def ParsePublicKeyPEM(data):
    """jwt/keyset.go:178-200 -> (PublicKey, err)."""
    try:
        return _h.parse_public_key_pem(data if isinstance(data, bytes) else data.encode()), None
    except ValueError as e:
        return None, str(e)


class KeySet:
    """jwt.KeySet (jwt/keyset.go:27-32), GPU-backed."""

    def __init__(self, impl):
        self._impl = impl

    def VerifySignature(self, token, ctx=None):
        return tuple(self._impl.verify_signature(token))

    def WaitTables(self):
        """Block until the key comb tables of the last key (re)load reach their
        budgeted width (keys verify before that, on narrower tables)."""
        self._impl.wait_tables()

    def VerifySignatureBatch(self, tokens: Sequence, ctx=None):
        return [tuple(r) for r in self._impl.verify_signature_batch(list(tokens))]

    def SetCoalescing(self, max_inflight=4, max_batch=65536, window_us=0):
        """Batching of concurrent single-token calls (VerifySignature and
        Validator.Validate): at most `max_inflight` device batches at once, each
        of at most `max_batch` tokens, collected for at most `window_us`.  The
        defaults are the library's (host/cap_jwt.hpp CoalesceConfig)."""
        self._impl.set_coalescing(int(max_inflight), int(max_batch), int(window_us))

    def CoalescingStats(self):
        return dict(self._impl.coalescing_stats())

    def DeviceStatus(self) -> str:
        """"" while the GPU context verifies; else why it is lost (it is
        recreated after a device error; see DeviceRecoveries)."""
        return self._impl.device_status()

    def DeviceRecoveries(self) -> int:
        return self._impl.device_recoveries()


def NewStaticKeySet(public_keys: List, devices=()):
    try:
        return KeySet(_h.new_static_keyset(list(public_keys), list(devices))), None
    except ValueError as e:
        return None, str(e)


def NewJSONWebKeySet(ctx, jwks_url: str, jwks_ca_pem: str = "", fetch: Callable = None, devices=()):
    try:
        return KeySet(_h.new_json_web_keyset(jwks_url, jwks_ca_pem, fetch, list(devices))), None
    except ValueError as e:
        return None, str(e)


def NewOIDCDiscoveryKeySet(ctx, issuer: str, issuer_ca_pem: str = "", fetch: Callable = None, devices=()):
    try:
        return KeySet(_h.new_oidc_discovery_keyset(issuer, issuer_ca_pem, fetch, list(devices))), None
    except ValueError as e:
        return None, str(e)


def _dur_ns(d) -> int:
    """time.Duration from a timedelta or a number of seconds."""
    if d is None:
        return 0
    if isinstance(d, datetime.timedelta):
        return (d.days * 86400 + d.seconds) * 1_000_000_000 + d.microseconds * 1000
    return int(round(d * 1e9))


def _time_ns(t) -> int:
    if isinstance(t, datetime.datetime):
        if t.tzinfo is None:
            t = t.replace(tzinfo=datetime.timezone.utc)
        d = t - datetime.datetime(1970, 1, 1, tzinfo=datetime.timezone.utc)
        return _dur_ns(d)
    return int(round(t * 1e9))


@dataclasses.dataclass
class Expected:
    """jwt/jwt.go:38-83.  Leeways: timedelta or seconds; Now: callable returning
    a datetime or unix seconds (None -> time.Now())."""
    Issuer: str = ""
    Subject: str = ""
    ID: str = ""
    Audiences: List[str] = dataclasses.field(default_factory=list)
    SigningAlgorithms: List[str] = dataclasses.field(default_factory=list)
    NotBeforeLeeway: object = 0
    ExpirationLeeway: object = 0
    ClockSkewLeeway: object = 0
    Now: Optional[Callable] = None

    def _native(self):
        e = _h.Expected()
        e.Issuer, e.Subject, e.ID = self.Issuer, self.Subject, self.ID
        e.Audiences = list(self.Audiences or [])
        e.SigningAlgorithms = list(self.SigningAlgorithms or [])
        e.NotBeforeLeeway = _dur_ns(self.NotBeforeLeeway)
        e.ExpirationLeeway = _dur_ns(self.ExpirationLeeway)
        e.ClockSkewLeeway = _dur_ns(self.ClockSkewLeeway)
        if self.Now is not None:
            e.has_now = True
            e.now_unix_ns = _time_ns(self.Now())
        return e


class Validator:
    """jwt.Validator (jwt/jwt.go:20-33)."""

    def __init__(self, keyset: KeySet):
        self._ks = keyset
        self._impl = _h.Validator(keyset._impl)

    def Validate(self, token, expected: Expected = None, ctx=None):
        return tuple(self._impl.validate(token, (expected or Expected())._native()))

    def ValidateBatch(self, tokens: Sequence, expected: Expected = None, ctx=None):
        """BASELINE north star: per-token result == Validate(tokens[i], expected)."""
        return [tuple(r) for r in self._impl.validate_batch(list(tokens), (expected or Expected())._native())]

    def ValidateBlob(self, blob: bytes, expected: Expected = None) -> bytes:
        """Newline-separated tokens -> one accept byte per token (throughput entry)."""
        return self._impl.validate_blob(blob, (expected or Expected())._native())


def NewValidator(keyset: Optional[KeySet]):
    if keyset is None:
        return None, "keySet must not be nil"
    return Validator(keyset), None


__all__ = ["RS256", "RS384", "RS512", "ES256", "ES384", "ES512", "PS256", "PS384", "PS512", "EdDSA",
           "DefaultLeewaySeconds", "PublicKey", "SupportedSigningAlgorithm", "ParsePublicKeyPEM", "KeySet",
           "NewStaticKeySet", "NewJSONWebKeySet", "NewOIDCDiscoveryKeySet", "Expected", "Validator", "NewValidator"]
