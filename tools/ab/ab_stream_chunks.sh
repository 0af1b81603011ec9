# configs[4] stream chunk-size sweep (run via gpurun from the repo root):
# bench.py --configs-only twice over a wider chunk list, ms per 1.25 M tokens
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sc
mkdir -p $O
for r in 1 2; do
  echo "== run $r $(date +%T)"
  timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 \
    --stream-chunks 196608,262144,327680,393216,458752,524288 > $O/c5_$r.json 2> $O/c5_$r.err || { echo C5_FAIL; tail -5 $O/c5_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$r.json'))['configs']['mixed_10alg_32kid']; s=d['stream']; print('resident', round(d['value']/1e6,2), 'stream', round(s['value']/1e6,2), {k: round(v,2) for k,v in s['ms_by_chunk'].items()})"
done
