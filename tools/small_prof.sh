# Phase timestamps of the one-launch small ECDSA kernel (k_ec_small built with
# JG_SMALL_PROF=1 into cap_amd/ab_sprof.so:
#   make -C cap_amd/csrc OBJDIR=build_ab/sprof OUT=../ab_sprof.so \
#        CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -DJG_SMALL_PROF=1" ../ab_sprof.so)
# run on the GPU box from the repo root; summary in gpurun_out/small_prof.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SBP_SIZES=1 CAPJWT_LIB="$GRAFT_REPO_ROOT/cap_amd/ab_sprof.so" timeout -k 10 200 \
  python3 -u tools/small_batch_probe.py gpurun_out/small_prof.json 1 ES256 > gpurun_out/small_prof.log 2>&1 || exit 1
python3 - <<'PY' > gpurun_out/small_prof.txt
import statistics
rows = []
for ln in open("gpurun_out/small_prof.log"):
    if ln.startswith("smallprof"):
        f = ln.split()
        rows.append([int(x) for x in f[2:10] + f[11:16]])
rows = rows[20:]
names = ["w0 staged", "w0 sig words", "w0 hash done", "w0 digits", "w0 point start", "w0 tree start",
         "w0 tree done", "w0 end", "w1 staged", "w1 sig words", "w1 inv+u2 done", "w1 digits done", "w1 phase6"]
for i, n in enumerate(names):
    print(f"{n:16s} {statistics.median(r[i] for r in rows) / 100:8.2f} us")
PY
cat gpurun_out/small_prof.txt
