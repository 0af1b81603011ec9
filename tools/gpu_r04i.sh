# Round-4 session I: configs[4] stream A/B over the class -> lane grouping
# (CAPJWT_CLASS_GROUP) and the plan-fill stream (CAPJWT_GROUP_CTRL).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grp
for spec in 0012222:least 0012222:copy 0012212:least 0102122:least 0102122:copy 0011222:least 0012222:least; do
  g=${spec%%:*}; c=${spec#*:}
  CAPJWT_CLASS_GROUP=$g CAPJWT_GROUP_CTRL=$c timeout -k 10 300 python -u tools/c5_stream_probe.py gpurun_out/grp/${g}_$c.json 4 524288 262144 > gpurun_out/grp/${g}_$c.txt 2>&1 || { echo "ST_FAIL $spec"; tail -30 gpurun_out/grp/${g}_$c.txt; exit 1; }
  echo "$spec: $(tr '\n' ' ' < gpurun_out/grp/${g}_$c.txt)"
done
