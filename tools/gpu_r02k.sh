# round-2 evidence after the RSA occupancy change: GPU parity suite, full bench, rocprofv3 passes,
# then the PS512 RSA-4096 probe A/B (default = modexp + PSS pad at 2 waves/SIMD; padw1 = pad at the
# compiler's occupancy; rsaw1 = both at the compiler's occupancy, the round-2 start)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/gpu_r02h.sh || exit 1
for v in default padw1 rsaw1 default padw1 rsaw1; do
  if [ $v = default ]; then lib=cap_amd/libcapjwt.so; else lib=cap_amd/ab_$v.so; fi
  CAPJWT_LIB=$lib timeout -k 10 300 python -u tools/config_probe.py ps512 > gpurun_out/ps512_$v.json 2> gpurun_out/ps512_$v.err || { echo PROBE_FAIL $v; tail -20 gpurun_out/ps512_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/ps512_$v.json)"
done
