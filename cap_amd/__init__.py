"""cap_amd -- MI355X-native batched JWS signature verification for hashicorp/cap's
jwt.KeySet / jwt.Validator path.  The product is libcapjwt.so
(include/jg.h); this package holds its Python binding and the Python mirror of
cap's jwt API."""
import os as _os

# tools/sanitize/run.sh: load an ASan/UBSan build of the host extension
# (_capjwt_host) from this directory instead of the regular one
if _os.environ.get("CAPJWT_HOST_EXT_DIR"):
    __path__.insert(0, _os.environ["CAPJWT_HOST_EXT_DIR"])

from . import _lib  # noqa: F401,E402
