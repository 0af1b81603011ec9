#!/bin/bash
# Run the host-layer CPU tests under ASan + UBSan (see Makefile).  CPU only.
#   bash tools/sanitize/run.sh [pytest args]
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
make -s -C "$HERE"
export CAPJWT_HOST_EXT_DIR="$HERE/build"
# python itself is not instrumented: preload the runtimes ahead of whatever
# the environment already preloads (kept as it is), and leave leak checking
# off (the interpreter's own arenas are never freed)
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)${LD_PRELOAD:+ $LD_PRELOAD}"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:strict_string_checks=1:detect_stack_use_after_return=1:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export CAPJWT_FUZZ_SCALE=${CAPJWT_FUZZ_SCALE:-10}
cd "$ROOT"
python3 -m pytest tests/test_host_cpu.py tests/test_oidc_hash.py -m "not gpu" -q -p no:cacheprovider "$@"
