"""cap_amd -- MI355X-native batched JWS signature verification for hashicorp/cap's
jwt.KeySet / jwt.Validator path.  The product is libcapjwt.so
(include/jg.h); this package holds its Python binding and the Python mirror of
cap's jwt API."""
from . import _lib  # noqa: F401
